# Ranged-read latency: separate keygen + split launches (XS_FUSED_MAX=0) vs the fused
# keygen+crypt launch for tiny zero-copy batches (default), alternating on one box; then
# kernel traces of both.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2 3; do
  for f in 0 16; do
    XS_FUSED_MAX=$f timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/fu_seek_f${f}_t1_$i.json
  done
done
for f in 0 16; do
  XS_FUSED_MAX=$f timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 > gpurun_out/fu_seek_f${f}_t16.json
  XS_FUSED_MAX=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fuprof_f$f -o run -- ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/fuprof_f$f.json
done
