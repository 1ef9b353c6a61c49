#!/bin/bash
# Round-4 refresh of the non-headline bench modes on the current tree: configs[2] (10 GiB of mixed
# objects with tag failures), configs[3] (1 TiB object set, generation + verification in the
# step), and file names with per-phase timing.
set -o pipefail
OUT=gpurun_out/${1:-r04_cfg}
mkdir -p $OUT
timeout -k 10 300 python bench.py --mixed-gib 10 --no-cpu > $OUT/mixed.json 2> $OUT/mixed.err || { echo MIXED_FAILED; tail $OUT/mixed.err; exit 1; }
cut -c1-400 $OUT/mixed.json
timeout -k 10 400 python bench.py --object-blocks 16777216 --steps 2 --warmup 1 --no-cpu > $OUT/objset.json 2> $OUT/objset.err || { echo OBJSET_FAILED; tail $OUT/objset.err; exit 1; }
cut -c1-400 $OUT/objset.json
RCLONE_AMD_NAME_TIMING=1 timeout -k 10 200 python bench.py --names 1000000 --no-cpu --steps 6 --warmup 2 > $OUT/names.json 2> $OUT/names.err || { echo NAMES_FAILED; tail $OUT/names.err; exit 1; }
tail -4 $OUT/names.err; cut -c1-300 $OUT/names.json
for b in 64 1024; do timeout -k 10 300 python tools/host_path_bench.py --batch $b >> $OUT/hostpath.json 2>>$OUT/hostpath.err || { echo HOSTPATH_FAILED; tail $OUT/hostpath.err; exit 1; }; done
cut -c1-300 $OUT/hostpath.json
echo CFG_DONE
