# Ranged-read latency: fused batches waited for by the event (XS_ENGINE_SPIN=0) vs by polling
# the kernel's completion word (default), alternating on one box.
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for v in 0 1; do
    XS_ENGINE_SPIN=$v timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/sp_seek_s${v}_t1_$i.json
  done
done
for v in 0 1; do
  XS_ENGINE_SPIN=$v timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 > gpurun_out/sp_seek_s${v}_t16.json
done
