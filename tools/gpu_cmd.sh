set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r02j.prof -- python3 $R/bench.py --no-cpu > $R/gpurun_out/r02j.prof.log 2>&1 || { echo PROF_FAILED; tail $R/gpurun_out/r02j.prof.log; exit 1; }
tail -1 $R/gpurun_out/r02j.prof.log | cut -c1-300
