# Ranged-read latency: fused kernel v1 (key schedule, then the four-wave split crypt) vs v2
# (key schedule on a fifth wave, overlapped with the keystream work; Poly1305 over LDS afterwards),
# alternating on one box; then kernel traces of both.  Output under gpurun_out/fv_*.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in 1 2; do
    XS_FUSED_V=$v timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/fv_seek_v${v}_t1_$i.json
  done
done
for v in 1 2; do
  XS_FUSED_V=$v timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 > gpurun_out/fv_seek_v${v}_t16.json
  XS_FUSED_V=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fvprof_v$v -o run -- ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/fvprof_v$v.json
done
echo fused_v_ab_done
