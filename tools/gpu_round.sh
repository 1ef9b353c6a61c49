#!/bin/bash
# One GPU session: full GPU tests, smoke, bench (1 GPU), host path, kernel trace profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$TAG.tests.log; exit 1; }
tail -2 gpurun_out/$TAG.tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/$TAG.smoke.log; exit 1; }
tail -1 gpurun_out/$TAG.smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { echo BENCH_FAILED; tail gpurun_out/$TAG.bench.err; exit 1; }
cat gpurun_out/$TAG.bench.json
for b in 64 256 1024; do timeout -k 10 300 python tools/host_path_bench.py --batch $b >> gpurun_out/$TAG.hostpath.json 2>>gpurun_out/$TAG.hostpath.err || exit 1; done
cat gpurun_out/$TAG.hostpath.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof -- python3 $R/bench.py --no-cpu > $R/gpurun_out/$TAG.prof.log 2>&1 || { echo PROF_FAILED; tail $R/gpurun_out/$TAG.prof.log; exit 1; }
tail -1 $R/gpurun_out/$TAG.prof.log
python3 $R/tools/prof_agree.py $R/gpurun_out/$TAG.prof $R/gpurun_out/$TAG.prof.log $R/gpurun_out/$TAG.timing_agreement.json
echo ROUND_DONE
