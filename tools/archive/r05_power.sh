#!/bin/bash
# Round 5: socket power and clocks while the bench line's steps run (read-only rocm-smi / amd-smi
# queries; nothing is set).  Evidence for "issue-bound at a power-limited clock": the package
# power against its cap while the shader clock sits below its maximum.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r05_power}
mkdir -p $OUT
timeout -k 5 20 rocm-smi --showpower --showmaxpower --showclocks > $OUT/idle_smi.txt 2>&1 || true
timeout -k 5 20 amd-smi metric --power --clock > $OUT/idle_amdsmi.txt 2>&1 || true
# a long headline run (300 steps, ~2 s) so the samples land inside the timed region
timeout -k 10 200 python3 bench.py --no-cpu --no-pool-check --objectset-steps 0 --steps 600 > $OUT/bench.json 2> $OUT/bench.err &
BP=$!
sleep 6
for i in $(seq 1 12); do
  date +%s.%N >> $OUT/load_smi.txt
  timeout -k 2 5 rocm-smi --showpower --showclocks >> $OUT/load_smi.txt 2>&1 || true
  sleep 0.3
done
wait $BP
rc=$?
cut -c1-250 $OUT/bench.json
grep -iE "power|sclk|fclk|mclk" $OUT/load_smi.txt | sort | uniq -c | sort -rn | head -20
exit $rc
