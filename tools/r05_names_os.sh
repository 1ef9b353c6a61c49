#!/bin/bash
# Round 5: the pipelined object-set pass and the pipelined names batches on the GPU -- their
# tests, the default bench line (configs[3] leg) and the names bench with per-call phases.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r05f}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest tests/test_objectset_gpu.py tests/test_dist_gpu.py tests/test_names_gpu.py -m gpu -x -v -s --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "PASSED|FAILED|ERROR" $OUT/tests.log | tail; tail -40 $OUT/tests.log; exit 1; }
grep -E "configs\[3\]" $OUT/tests.log; tail -1 $OUT/tests.log
timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail $OUT/bench.err; exit 1; }
cut -c1-200 $OUT/bench.json
RCLONE_AMD_NAME_TIMING=1 timeout -k 10 300 python3 bench.py --names 1000000 --steps 10 --warmup 3 > $OUT/names.json 2> $OUT/names_phases.txt || { echo NAMES_FAILED; tail $OUT/names_phases.txt; exit 1; }
cut -c1-300 $OUT/names.json
tail -4 $OUT/names_phases.txt
echo R05F_DONE
