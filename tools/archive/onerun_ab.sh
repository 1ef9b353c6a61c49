#!/bin/bash
# One (direction, key) run per combined batch (XS_BATCH_ONE_RUN=1) vs mixed batches (0):
# many-handle encrypt + decrypt streams (coalesce_bench, 16 threads) at 64 KiB, 1 MiB and 8 MiB,
# and the engine GPU tests with the option on; alternating on one box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
OUT=gpurun_out/onerun_ab.jsonl
: > $OUT
for i in 1 2 3; do
  for v in 0 1; do
    for ob in "800 65536" "100 1048576" "16 8388608"; do
      set -- $ob
      r=$(XS_BATCH_ONE_RUN=$v timeout -k 10 60 ./tools/coalesce_bench 16 $1 $2 1) || { echo BENCH_FAILED; exit 1; }
      echo "{\"one_run\": $v, \"run\": $i, \"cb\": $r}" >> $OUT
    done
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/onerun_ab.jsonl"):
    r = json.loads(l)
    d[(r["cb"]["object_bytes"], r["one_run"])].append(r["cb"]["GiB_s"])
for k in sorted(d): print(k, d[k])
PY
XS_BATCH_ONE_RUN=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_engine_coalesce_gpu.py tests/test_cipher_gpu.py tests/test_fused_gpu.py > gpurun_out/onerun_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/onerun_tests.log; exit 1; }
tail -1 gpurun_out/onerun_tests.log
