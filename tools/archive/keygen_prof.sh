# Kernel durations of the ranged-read path with the narrow (one lane per block) and the wide
# (one wave per block) keygen: rocprofv3 kernel-trace stats of tools/seek_latency.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for w in 0 16; do
  XS_KEYGEN_WIDE_MAX=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kgprof_w$w -o run -- ./tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > gpurun_out/kgprof_w$w.json
done
