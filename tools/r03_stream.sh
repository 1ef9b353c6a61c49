#!/bin/bash
# round-3 GPU session: new per-object hash tests, then configs[4] stream shapes at 16 GiB (A/B of
# the tee placement and MD5 workers).  Every GPU step under its own time limit, chained with &&.
set -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_hash_stream_gpu.py tests/test_cryptfs_gpu.py tests/test_md5_gpu.py > $OUT/tests_new.log 2>&1 || { echo tests_failed; tail -30 $OUT/tests_new.log; exit 1; }
tail -3 $OUT/tests_new.log
D=/dev/shm/rc_e2e_r03
run() { timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D "$@" >> $OUT/e2e16.jsonl 2>> $OUT/e2e16.err; }
run --mode stream --transfers 4 --check-mode stream --checkers 8 &&
run --mode stream --transfers 4 --tee reader --check-mode stream --checkers 8 &&
XS_MD5_WORKERS=0 run --mode stream --transfers 4 --check-mode stream --checkers 8 &&
run --mode stream --transfers 16 --check-mode stream --checkers 16 &&
run --lanes 4 --transfers 16 || { echo e2e_failed; cat $OUT/e2e16.err | tail; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r03b/e2e16.jsonl"):
    r = json.loads(l)
    print(r["mode"], r["tee"], r["check_mode"], r["transfers"], r["checkers"], "sync", r["sync_GiB_s"], "check", r["cryptcheck_GiB_s"], "ok", r["ok"])
PY
