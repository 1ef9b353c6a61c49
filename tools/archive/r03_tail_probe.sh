#!/bin/bash
# Grid-tail probe: seal/open kernel time per block at 98 304 blocks (exactly 24 rounds of the
# 4096 resident waves) vs 100 000 (24.4 rounds), alternating.
set -o pipefail
OUT=gpurun_out/${1:-r03_tail}
mkdir -p $OUT
for i in 1 2; do for nb in 98304 100000 102400; do
  timeout -k 10 200 python3 bench.py --blocks $nb --no-cpu --steps 40 > $OUT/b_$nb.json 2>> $OUT/err.txt || { echo FAIL; tail $OUT/err.txt; exit 1; }
  python3 -c "
import json; r=json.load(open('$OUT/b_$nb.json')); ro=r['roofline']
print(json.dumps({'blocks': $nb, 'seal_ms': ro['kernel_ms_avg'], 'open_ms': ro['open']['kernel_ms_avg'], 'seal_us_per_kblock': ro['kernel_ms_avg']/$nb*1e6, 'open_us_per_kblock': ro['open']['kernel_ms_avg']/$nb*1e6, 'clock': (r.get('clock') or {}).get('shader_clock_ghz')}))" | tee -a $OUT/tail.jsonl
done; done
