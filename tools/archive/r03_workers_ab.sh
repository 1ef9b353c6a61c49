#!/bin/bash
# Per-object shapes at 16 GiB: MD5 worker count (inline fallback when all are busy), at the
# reference defaults and at 16 transfers / checkers.
set -o pipefail
OUT=gpurun_out/${1:-r03_workers}
mkdir -p $OUT
D=/dev/shm/rc_e2e_w
run() { timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D --mode stream --check-mode stream "$@" >> $OUT/e2e16.jsonl 2>> $OUT/e2e16.err; }
for w in 8 16 0; do
  XS_MD5_WORKERS=$w run --transfers 16 --checkers 16 &&
  XS_MD5_WORKERS=$w run --transfers 4 --checkers 8 || { echo E2E_FAILED; tail $OUT/e2e16.err; rm -rf $D; exit 1; }
done
rm -rf $D
python3 - $OUT <<'PY'
import json, sys
for l in open(sys.argv[1] + "/e2e16.jsonl"):
    r = json.loads(l)
    print(r["transfers"], r["checkers"], "sync", r["sync_GiB_s"], "check", r["cryptcheck_GiB_s"], "ok", r["ok"])
PY
