#!/bin/bash
# File names: the names GPU tests, then bench.py --names with the pipelined name batches on (4
# parts) vs off (RCLONE_AMD_NAME_PIPE=1: every host stage, then one launch), alternating.
set -o pipefail
OUT=gpurun_out/${1:-r03_names_pipe}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_names_gpu.py > $OUT/names_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/names_tests.log; exit 1; }
tail -1 $OUT/names_tests.log
for i in $(seq ${PAIRS:-4}); do for g in ${ORDER:-4 1}; do
  RCLONE_AMD_NAME_PIPE=$g timeout -k 10 200 python bench.py --names 1000000 --no-cpu --steps 20 --warmup 5 > $OUT/n.json 2> $OUT/n.err || { echo BENCH_FAILED; tail $OUT/n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/n.json')); print(json.dumps({'parts': $g, 'names_per_s': d['value'], 'encrypt_s': d['encrypt_s'], 'decrypt_s': d['decrypt_s']}))" | tee -a $OUT/names_ab.jsonl
done; done
