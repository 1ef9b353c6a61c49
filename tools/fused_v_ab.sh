# Ranged-read latency, paired on one box: fused v2 (four crypt waves + key wave) vs v3 (eight
# crypt waves, two per SIMD, + key wave), 1 and 16 readers, alternating; kernel traces of both;
# per-wave phase marks of v3 (tools/fused_probe).  Output under gpurun_out/fv_*.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in 2 3; do
    XS_FUSED_V=$v timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/fv_seek_v${v}_t1_$i.json
    XS_FUSED_V=$v timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 > gpurun_out/fv_seek_v${v}_t16_$i.json
  done
done
for v in 2 3; do
  XS_FUSED_V=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fvprof_v$v -o run -- ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/fvprof_v$v.json
done
timeout -k 10 60 ./tools/fused_probe 200 1 8 1 > gpurun_out/fv_probe_v3.json
timeout -k 10 60 ./tools/fused_probe 200 1 4 1 > gpurun_out/fv_probe_v2.json
echo fused_v_ab_done
