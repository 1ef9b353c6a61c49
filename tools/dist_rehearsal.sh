# Multi-rank rehearsal on a one-GPU box: bench.py --gpus N starts its own N ranks (gloo, sharing
# the GPU) in every mode; each line must carry n_gpus = ranks_seen = N.  The same checks run in
# the -m gpu suite (tests/test_dist_gpu.py); this script keeps the full-size lines.
set -o pipefail
mkdir -p gpurun_out
export BENCH_DIST_BACKEND=gloo
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/$name.json 2> gpurun_out/$name.err || { echo FAIL $name; tail -30 gpurun_out/$name.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/$name.json').read().strip().splitlines()[-1]); c=d['config']
assert d['n_gpus']==c['ranks_seen'], d
k=d.get('counters') or {}; o=d.get('objectset') or {}
assert k.get('tag_digest_ok', True) and o.get('ok', True), (k, o)
print('$name', d['value'], d['unit'], 'ranks_seen', c['ranks_seen'], 'distinct_gpus', c['distinct_gpus'],
      'digest', k.get('tag_digest'), 'expected', k.get('tag_digest_expected'), 'objectset', o.get('value'), o.get('ok'))"
}
run dist2 --gpus 2 --steps 3 --warmup 2
run dist4 --gpus 4 --steps 3 --warmup 2 --blocks 50000
run dist2_obj --gpus 2 --steps 2 --warmup 1 --object-blocks 400000
run dist2_names --gpus 2 --steps 2 --warmup 1 --names 200000
# the driver's N = 8 shape, eight gloo ranks on the one GPU: the headline set at 100 000 blocks per
# rank (its 800 000-block digest is pinned by the CPU oracle, tests/golden/fullsize.json), then the
# configs[3] leg at world 8 (smaller headline share so eight ranks' buffers fit one GPU's HBM)
if [ -n "$DIST8" ]; then
  run dist8 --gpus 8 --steps 2 --warmup 1 --warmup-seconds 0 --objectset-steps 0 --no-pool-check
  BENCH_OBJECTSET_ROUND_BLOCKS=50000 run dist8_objset --gpus 8 --steps 2 --warmup 1 --warmup-seconds 0 --blocks 20000 --objectset-steps 1 --objectset-warmup 0 --no-pool-check
fi
echo REHEARSAL_DONE
