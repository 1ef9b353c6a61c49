# ARCHIVED (round 6): ran the keygen-overlap A/B against a bench.py variant with BENCH_KEYGEN_SERIAL,
# which was not kept (profiles/r06/keygen_overlap_ab/).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/r06s; mkdir -p $OUT
for rep in 1 2 3; do
  for v in overlap serial; do
    if [ $v = serial ]; then export BENCH_KEYGEN_SERIAL=1; else unset BENCH_KEYGEN_SERIAL; fi
    timeout -k 10 200 python3 bench.py --no-cpu --no-pool-check --objectset-steps 0 --steps 200 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b.json')); r=d['roofline']
print(json.dumps({'v': '$v', 'rep': $rep, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'seal_ms': r['kernel_ms_avg'], 'open_ms': r['open']['kernel_ms_avg'], 'clock': d['clock']['shader_clock_ghz'], 'digest_ok': d['counters']['tag_digest_ok'], 'J_per_GiB': d['energy_J_per_GiB']}))" >> $OUT/ab.jsonl
  done
done
cat $OUT/ab.jsonl
