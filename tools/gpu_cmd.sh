set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 500 --timeout-method thread -p no:cacheprovider tests/test_fused_gpu.py tests/test_engine_coalesce_gpu.py tests/test_cipher_gpu.py tests/test_gpu_parity.py > gpurun_out/r02ba.tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02ba.tests.log; exit 1; }
tail -1 gpurun_out/r02ba.tests.log
