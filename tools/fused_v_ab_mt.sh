# Ranged-read throughput under concurrency: fused v1 vs v2, alternating, 4 and 16 reader threads,
# then kernel traces at 16 threads.  Output under gpurun_out/fvmt_*.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do
  for t in 4 16; do
    for v in 1 2; do
      XS_FUSED_V=$v timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads $t > gpurun_out/fvmt_v${v}_t${t}_$i.json
    done
  done
done
for v in 1 2; do
  XS_FUSED_V=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fvmtprof_v$v -o run -- ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 > gpurun_out/fvmtprof_v$v.json
done
echo fused_v_ab_mt_done
