# Express lanes A/B: off (XS_EXPRESS_MAX=0) vs 1, 2, 4 lanes (XS_EXPRESS_LANES): many-handle
# streaming throughput with the reference-like first refill of one block (read-ahead 1), full
# first batches (read-ahead 0) for reference, and ranged reads; alternating on one box.
# Output: gpurun_out/ex_*.jsonl
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for cfg in "0 1" "4 1" "4 2" "4 4"; do
    set -- $cfg
    x=$1; n=$2
    for ob in "800 65536" "16 8388608"; do
      set -- $ob
      XS_EXPRESS_MAX=$x XS_EXPRESS_LANES=$n timeout -k 10 60 ./tools/coalesce_bench 16 $1 $2 1 >> gpurun_out/ex_cb_x${x}_n${n}.jsonl
    done
    XS_EXPRESS_MAX=$x XS_EXPRESS_LANES=$n timeout -k 10 60 ./tools/coalesce_bench 16 16 8388608 0 >> gpurun_out/ex_cb_x${x}_n${n}.jsonl
    XS_EXPRESS_MAX=$x XS_EXPRESS_LANES=$n timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 >> gpurun_out/ex_seek_x${x}_n${n}.jsonl
  done
done
echo express_ab_done
