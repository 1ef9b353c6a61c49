set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_readahead_gpu.py tests/test_cipher_gpu.py > gpurun_out/r02d.tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02d.tests.log; exit 1; }
tail -3 gpurun_out/r02d.tests.log
rm -f gpurun_out/r02d.coalesce.jsonl
for rep in 1 2 3; do for S in 65536 1048576 8388608; do for ra in 1 0; do
  K=$((800*65536/S)); [ $K -lt 16 ] && K=16
  timeout -k 10 120 ./tools/coalesce_bench 16 $K $S $ra >> gpurun_out/r02d.coalesce.jsonl || exit 1
done; done; done
cat gpurun_out/r02d.coalesce.jsonl
