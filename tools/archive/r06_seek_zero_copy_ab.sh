set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/r06v
for rep in 1 2; do for zc in 1 0; do
  XS_ENGINE_ZERO_COPY=$zc timeout -k 5 120 ./tools/seek_latency --mib 256 --reads 64000 --len 4096 --threads 16 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['zero_copy']=$zc; print(json.dumps(d))" >> gpurun_out/r06v/zc.jsonl || exit 1
done; done
python3 -c "
import json
for l in open('gpurun_out/r06v/zc.jsonl'):
    d=json.loads(l); print('zc', d['zero_copy'], 'p50', d['p50_us'], 'reads/s', d['reads_per_s'], 'req/batch', round(d['engine_requests']/max(1,d['engine_batches']),2))"
