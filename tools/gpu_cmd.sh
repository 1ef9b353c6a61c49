set -o pipefail
mkdir -p gpurun_out
bash tools/fused_v_ab_mt.sh > gpurun_out/fvmt.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/fvmt.log; exit 1; }
for f in gpurun_out/fvmt_*.json gpurun_out/fvmtprof_*.json; do echo $f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['p50_us'], d['p99_us'], d['reads_per_s'], d['bad'])"); done
