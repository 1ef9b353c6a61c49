#!/bin/bash
# 16 concurrent ranged 4 KiB readers on the GPU engine under its concurrency knobs:
# express lanes, express size limit, spin waiting, ring slots -- alternated twice.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-seek_knobs}
mkdir -p $OUT
T=${THREADS:-16}
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 5 120 ./tools/seek_latency --mib 256 --reads $((4000 * T)) --len 4096 --threads $T > $OUT/tmp.json || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/tmp.json').read().strip().splitlines()[-1]); d['label']='$label'; print(json.dumps(d))" >> $OUT/knobs.jsonl
}
if [ -z "$SET2" ]; then
for rep in 1 2; do
  run default
  run lanes4 XS_EXPRESS_LANES=4
  run lanes8 XS_EXPRESS_LANES=8
  run lanes0 XS_EXPRESS_MAX=0
  run nospin XS_ENGINE_SPIN=0
  run slots6 RCLONE_AMD_ENGINE_SLOTS=6
  run lanes8_nospin XS_EXPRESS_LANES=8 XS_ENGINE_SPIN=0
done
else  # the ring's shape: fewer slots (bigger combined batches), issue-while-waiting, wake-all
for rep in 1 2; do
  run default
  run slots1 RCLONE_AMD_ENGINE_SLOTS=1
  run slots2 RCLONE_AMD_ENGINE_SLOTS=2
  run overlap XS_ENGINE_OVERLAP=1
  run overlap_slots2 XS_ENGINE_OVERLAP=1 RCLONE_AMD_ENGINE_SLOTS=2
  run wakeall XS_ENGINE_WAKE_ALL=1
  run lanes0_slots2 XS_EXPRESS_MAX=0 RCLONE_AMD_ENGINE_SLOTS=2
done
fi
python3 -c "
import json
for l in open('$OUT/knobs.jsonl'):
    d = json.loads(l); print(d['label'], 'p50', d['p50_us'], 'p99', d['p99_us'], 'reads/s', d['reads_per_s'],
                             'req/batch', round(d.get('engine_requests', 0) / max(1, d.get('engine_batches', 1)), 2))
"
