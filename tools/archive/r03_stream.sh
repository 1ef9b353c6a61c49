#!/bin/bash
# round-3 GPU session: the whole -m gpu suite, then configs[4] stream shapes at 16 GiB (A/B of the
# tee placement and MD5 workers).  Every GPU step under its own time limit, chained with &&.
set -o pipefail
OUT=gpurun_out/${R03_TAG:-r03b}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests_failed; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> $OUT/gpu_tests.log 2>&1 || { echo smoke_failed; tail -20 $OUT/gpu_tests.log; exit 1; }
D=/dev/shm/rc_e2e_r03
run() { timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D "$@" >> $OUT/e2e16.jsonl 2>> $OUT/e2e16.err; }
run --mode stream --transfers 4 --check-mode stream --checkers 8 &&
run --mode stream --transfers 4 --tee reader --check-mode stream --checkers 8 &&
XS_MD5_WORKERS=0 run --mode stream --transfers 4 --check-mode stream --checkers 8 &&
run --mode stream --transfers 16 --check-mode stream --checkers 16 &&
run --lanes 4 --transfers 16 || { echo e2e_failed; tail $OUT/e2e16.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
for l in open(sys.argv[1] + "/e2e16.jsonl"):
    r = json.loads(l)
    print(r["mode"], r["tee"], r["check_mode"], r["transfers"], r["checkers"], "sync", r["sync_GiB_s"], "check", r["cryptcheck_GiB_s"], "ok", r["ok"])
PY
