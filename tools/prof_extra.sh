#!/bin/bash
# rocprofv3 kernel traces of the secondary bench modes (configs[2] mixed objects, file names).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mixed -- python3 $R/bench.py --mixed-gib 10 --steps 10 --warmup 3 --no-cpu > $R/gpurun_out/prof_mixed.log 2>&1 || { echo MIXED_FAILED; tail $R/gpurun_out/prof_mixed.log; exit 1; }
grep '^{' $R/gpurun_out/prof_mixed.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_names -- python3 $R/bench.py --names 1000000 --steps 5 --warmup 2 --no-cpu > $R/gpurun_out/prof_names.log 2>&1 || { echo NAMES_FAILED; tail $R/gpurun_out/prof_names.log; exit 1; }
grep '^{' $R/gpurun_out/prof_names.log
echo PROF_EXTRA_DONE
