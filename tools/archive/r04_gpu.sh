#!/bin/bash
# Round-4 GPU session: the whole -m gpu suite, smoke, the bench line (N=1), the self-launched
# 2-rank bench (gloo ranks sharing the box's GPU), optionally the kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04a}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "PASSED|FAILED|ERROR|configs\[4\]" $OUT/gpu_tests.log | tail -20; tail -60 $OUT/gpu_tests.log; exit 1; }
grep -E "^configs\[4\] (batch|stream):" $OUT/gpu_tests.log
tail -1 $OUT/gpu_tests.log
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail $OUT/bench.err; exit 1; }
cut -c1-600 $OUT/bench.json
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --no-cpu > $OUT/bench2.json 2> $OUT/bench2.err || { echo BENCH2_FAILED; tail $OUT/bench2.err; exit 1; }
cut -c1-400 $OUT/bench2.json
if [ -n "$PROF" ]; then
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -- python3 $R/bench.py --no-cpu > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail $OUT/prof.log; exit 1; }
cd $R && python3 tools/prof_agree.py $OUT/prof $OUT/prof.log $OUT/timing_agreement.json > /dev/null 2>&1 || echo prof_agree_failed
fi
echo R04_DONE
