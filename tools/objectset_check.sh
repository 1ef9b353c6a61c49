set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider tests/test_objectset_gpu.py > gpurun_out/objset_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/objset_tests.log; exit 1; }
tail -1 gpurun_out/objset_tests.log
timeout -k 10 300 python bench.py --object-blocks 16777216 --steps 2 --warmup 1 > gpurun_out/objset_bench.json 2> gpurun_out/objset_bench.err || { echo BENCH_FAILED; tail gpurun_out/objset_bench.err; exit 1; }
cat gpurun_out/objset_bench.json
