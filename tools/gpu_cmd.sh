set -o pipefail
mkdir -p gpurun_out
for t in 1 4; do for bb in 64 256; do
  echo "threads $t batch $bb: $(timeout -k 10 60 ./tools/coalesce_bench $t 32 8388608 0 $bb | cut -c1-200)"
  echo "threads $t batch $bb 64MiB: $(timeout -k 10 60 ./tools/coalesce_bench $t 8 67108864 0 $bb | cut -c1-200)"
done; done
