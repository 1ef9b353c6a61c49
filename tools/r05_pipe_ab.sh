#!/bin/bash
# Round 5 paired A/B on one box: object-set pass pipelined vs stream order (configs[3], 1 TiB,
# 3 steps), and names batches in 4 pipelined groups vs one group (1 M names), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05g}
mkdir -p $OUT
cd $R
for i in 1 2 3; do
  for p in 1 0; do
    BENCH_OBJECTSET_PIPELINE=$p timeout -k 10 200 python3 bench.py --object-blocks 16777216 --steps 3 --warmup 1 > $OUT/os_p${p}_$i.json 2> $OUT/os_p${p}_$i.err || { echo OS_FAILED; tail $OUT/os_p${p}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('objectset pipeline=$p', d['value'], d['ms_per_step'], d['counters']['tag_digest'])" $OUT/os_p${p}_$i.json
  done
  for g in 32 1000; do
    RCLONE_AMD_NAME_GROUP_CHUNKS=$g timeout -k 10 200 python3 bench.py --names 1000000 --steps 10 --warmup 3 > $OUT/names_g${g}_$i.json 2> $OUT/names_g${g}_$i.err || { echo NAMES_FAILED; tail $OUT/names_g${g}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('names groups_of=$g', d['value'], d['encrypt_s'], d['decrypt_s'])" $OUT/names_g${g}_$i.json
  done
done
echo AB_DONE
