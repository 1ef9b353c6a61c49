#!/bin/bash
# Per-object shapes at 16 GiB: worker MD5 rate in context (RCLONE_AMD_PHASES md5_worker_GB_s) and
# the cgroup's CPU throttling, for a knob ABVAR (values A B, alternating, PAIRS times).
set -o pipefail
OUT=gpurun_out/${1:-r03_spin}
ABVAR=${ABVAR:-XS_ENGINE_SPIN}; A=${A:-1}; B=${B:-0}
mkdir -p $OUT
for i in $(seq ${PAIRS:-2}); do for s in $A $B; do
  echo "$ABVAR=$s before $(tr '\n' ' ' < /sys/fs/cgroup/cpu.stat)" >> $OUT/cpustat.txt
  env $ABVAR=$s RCLONE_AMD_PHASES=1 timeout -k 10 300 tools/e2e_sync --gib 16 --dir /dev/shm/rc_sp --mode stream --check-mode stream --transfers 4 --checkers 8 > $OUT/e2e_$s.json 2> $OUT/phases_$s.txt || { echo FAIL; rm -rf /dev/shm/rc_sp; exit 1; }
  echo "$ABVAR=$s after $(tr '\n' ' ' < /sys/fs/cgroup/cpu.stat)" >> $OUT/cpustat.txt
  python3 -c "
import json,sys
r=json.load(open('$OUT/e2e_$s.json')); p=json.loads(open('$OUT/phases_$s.txt').read().strip().splitlines()[-1])['rclone_amd_phases']
print('$ABVAR', '$s', 'sync', r['sync_GiB_s'], 'check', r['cryptcheck_GiB_s'], 'md5_worker_GB_s', p['md5_worker_GB_s'])" | tee -a $OUT/summary.txt
done; done
rm -rf /dev/shm/rc_sp
