set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/spin_*.txt
for i in 1 2; do for sp in 200 30 10; do for t in 1 4 16; do
  echo "$sp $(XS_SPIN_PURE_US=$sp timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads $t | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['threads'], d['p50_us'], d['p99_us'], d['reads_per_s'], d['mean_open_us'], d['mean_read_us'], d['bad'])")" | tee -a gpurun_out/spin_ab.txt || exit 1
done; XS_SPIN_PURE_US=$sp timeout -k 10 30 ./tools/engine_rate 16 2 | tee -a gpurun_out/spin_ab.txt; done; done
