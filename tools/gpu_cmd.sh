set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/fv_* gpurun_out/fvprof_*
timeout -k 10 900 python -u -m pytest -x -q --timeout 500 --timeout-method thread -p no:cacheprovider tests/test_fused_gpu.py tests/test_gpu_parity.py tests/test_engine_coalesce_gpu.py tests/test_cipher_gpu.py > gpurun_out/r02ah.tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02ah.tests.log; exit 1; }
tail -2 gpurun_out/r02ah.tests.log
bash tools/fused_v_ab.sh > gpurun_out/fv_ab.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/fv_ab.log; exit 1; }
for f in gpurun_out/fv_seek_*.json; do echo $f $(python3 -c "import json; d=json.load(open('$f')); print(d['p50_us'], d['p90_us'], d['p99_us'], d['reads_per_s'], d['bad'])"); done
