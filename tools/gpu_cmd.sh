set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider -k "independent or full_size" > gpurun_out/r02x.tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02x.tests.log; exit 1; }
tail -3 gpurun_out/r02x.tests.log
timeout -k 10 300 python3 bench.py --independent --cpu-seconds 2 > gpurun_out/bench_r02x_indep.json 2> gpurun_out/bench_r02x_indep.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_r02x_indep.err; exit 1; }
tail -1 gpurun_out/bench_r02x_indep.json | cut -c1-700
