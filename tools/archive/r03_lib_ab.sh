#!/bin/bash
# Per-object shapes at 16 GiB, the current library vs another build of it (tools/ab_old/: the
# library and an e2e_sync_old linked to it with RUNPATH $ORIGIN), alternating; with the worker
# MD5 rate in context (RCLONE_AMD_PHASES md5_worker_GB_s).
set -o pipefail
OUT=gpurun_out/${1:-r03_lib}
mkdir -p $OUT
for i in $(seq ${PAIRS:-3}); do for v in new old; do
  if [ $v = old ]; then E=tools/ab_old/e2e_sync_old; else E=tools/e2e_sync; fi
  RCLONE_AMD_PHASES=1 timeout -k 10 300 $E --gib 16 --dir /dev/shm/rc_ab --mode stream \
    --check-mode stream --transfers ${TR:-4} --checkers ${CK:-8} > $OUT/e2e_$v.json 2> $OUT/phases_$v.txt || { echo FAIL; tail $OUT/phases_$v.txt; rm -rf /dev/shm/rc_ab; exit 1; }
  python3 -c "
import json
r=json.load(open('$OUT/e2e_$v.json')); p=json.loads(open('$OUT/phases_$v.txt').read().strip().splitlines()[-1])['rclone_amd_phases']
r['lib']='$v'; r['md5_worker_GB_s']=p.get('md5_worker_GB_s')
print(json.dumps(r))" >> $OUT/e2e16.jsonl
done; done
rm -rf /dev/shm/rc_ab
python3 - $OUT <<'PY'
import json, sys
for l in open(sys.argv[1] + "/e2e16.jsonl"):
    r = json.loads(l)
    print(r["lib"], r["transfers"], r["checkers"], "sync", r["sync_GiB_s"], "check", r["cryptcheck_GiB_s"], "md5_worker_GB_s", r["md5_worker_GB_s"], "ok", r["ok"])
PY
