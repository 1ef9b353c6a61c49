set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python3 bench.py > gpurun_out/bench_r02v_$i.json 2> gpurun_out/bench_r02v_$i.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_r02v_$i.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r02v_$i.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['open']['kernel_ms_avg'], d['clock'], d['cpu_baseline'])"
done
