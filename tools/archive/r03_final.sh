#!/bin/bash
# Round-3 closing GPU session: the whole -m gpu suite, smoke, the bench line, and its kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r03z}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -- python3 $R/bench.py --no-cpu > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail $OUT/prof.log; exit 1; }
cd $R && python3 tools/prof_agree.py $OUT/prof $OUT/prof.log $OUT/timing_agreement.json > /dev/null 2>&1 || echo prof_agree_failed
echo FINAL_DONE
