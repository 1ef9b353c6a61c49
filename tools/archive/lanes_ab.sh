#!/bin/bash
# Express lanes per engine (XS_EXPRESS_LANES): 2 (default) vs 3 vs 4, with one (direction, key) run
# per ring batch -- many-handle streams (coalesce_bench, 16 threads) and 16 concurrent ranged readers;
# alternating on one box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
OUT=gpurun_out/lanes_ab.jsonl
: > $OUT
for i in 1 2 3; do
  for v in 2 3 4; do
    for ob in "800 65536" "100 1048576" "16 8388608"; do
      set -- $ob
      r=$(XS_EXPRESS_LANES=$v timeout -k 10 60 ./tools/coalesce_bench 16 $1 $2 1) || { echo BENCH_FAILED; exit 1; }
      echo "{\"lanes\": $v, \"run\": $i, \"cb\": $r}" >> $OUT
    done
    r=$(XS_EXPRESS_LANES=$v timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16) || { echo SEEK_FAILED; exit 1; }
    echo "{\"lanes\": $v, \"run\": $i, \"seek\": $r}" >> $OUT
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/lanes_ab.jsonl"):
    r = json.loads(l)
    if "cb" in r: d[("cb", r["cb"]["object_bytes"], r["lanes"])].append(r["cb"]["GiB_s"])
    else: d[("seek", r["lanes"])].append({k: r["seek"][k] for k in r["seek"] if k in ("reads_per_s", "p50_us", "p99_us")})
for k in sorted(d, key=str): print(k, d[k])
PY
