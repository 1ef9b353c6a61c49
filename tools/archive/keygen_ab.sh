set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/kg_parity.log 2>&1
for i in 1 2 3; do
  for w in 0 16; do
    XS_KEYGEN_WIDE_MAX=$w timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/kg_seek_w${w}_t1_$i.json
  done
done
for w in 0 16; do
  XS_KEYGEN_WIDE_MAX=$w timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 > gpurun_out/kg_seek_w${w}_t16.json
done
