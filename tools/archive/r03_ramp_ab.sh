#!/bin/bash
# Per-object shapes at 16 GiB with a knob on vs off, alternating: ABVAR, default the MD5 ramp
# (RCLONE_AMD_MD5_RAMP, cipher.cpp; XS_MD5_CHAIN for job chaining, md5_workers.h), plus the
# aggregate MD5 rate of T concurrent host streams (tools/microbench/md5_threads: the ceiling of a
# shape with T transfers or checkers; NOTHREADS=1 skips it).
set -o pipefail
OUT=gpurun_out/${1:-r03_ramp}
PAIRS=${2:-3}
mkdir -p $OUT
[ -n "$NOTHREADS" ] || timeout -k 5 90 tools/microbench/md5_threads 1.5 1 2 4 8 12 16 > $OUT/md5_threads.jsonl || { echo MD5_THREADS_FAILED; exit 1; }
D=/dev/shm/rc_e2e_r
run() {  # ramp transfers checkers
  env ${ABVAR:-RCLONE_AMD_MD5_RAMP}=$1 timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D --mode stream --check-mode stream \
    --check-dst-hash ${DSTHASH:-1} --transfers $2 --checkers $3 > $OUT/one.json 2>> $OUT/e2e16.err &&
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); r[sys.argv[3]]=int(sys.argv[2]); print(json.dumps(r))" \
    $OUT/one.json $1 ${ABVAR:-RCLONE_AMD_MD5_RAMP} >> $OUT/e2e16.jsonl
}
for i in $(seq $PAIRS); do
  for r in 1 0; do
    run $r 4 8 || { echo E2E_FAILED; tail $OUT/e2e16.err; rm -rf $D; exit 1; }
  done
done
for i in $(seq ${PAIRS16:-2}); do
  for r in 1 0; do
    run $r 16 16 || { echo E2E_FAILED; tail $OUT/e2e16.err; rm -rf $D; exit 1; }
  done
done
RCLONE_AMD_PHASES=1 timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D --mode stream \
  --check-mode stream --transfers 4 --checkers 8 > $OUT/phases_ramp1.json 2> $OUT/phases_ramp1.txt ||
  { echo PHASES_FAILED; rm -rf $D; exit 1; }
rm -rf $D
cat $OUT/md5_threads.jsonl
python3 - $OUT <<'PY'
import json, sys
for l in open(sys.argv[1] + "/e2e16.jsonl"):
    r = json.loads(l)
    k = [x for x in r if x.startswith(("RCLONE_AMD", "XS_"))][0]
    print(k, r[k], r["transfers"], r["checkers"], "sync", r["sync_GiB_s"], "check", r["cryptcheck_GiB_s"], "ok", r["ok"])
PY
tail -1 $OUT/phases_ramp1.txt
