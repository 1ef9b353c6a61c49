#!/bin/bash
# Paired A/B of the names path: this tree vs tools/abprev (an older tree built in place),
# alternating on one box; then the names GPU tests on this tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/names_ab.jsonl
mkdir -p $R/gpurun_out
: > $OUT
for i in 1 2 3; do
  for side in new old; do
    d=$R; [ $side = old ] && d=$R/tools/abprev
    (cd $d && timeout -k 10 200 python bench.py --names 1000000 --no-cpu --steps 20 --warmup 5) > /tmp/n.json 2>/tmp/n.err || { echo BENCH_FAILED $side; tail /tmp/n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('/tmp/n.json')); print(json.dumps({'side':'$side','run':$i,'names_per_s':d['value'],'encrypt_s':d['encrypt_s'],'decrypt_s':d['decrypt_s']}))" | tee -a $OUT
  done
done
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_names_gpu.py > gpurun_out/names_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/names_tests.log; exit 1; }
tail -1 gpurun_out/names_tests.log
