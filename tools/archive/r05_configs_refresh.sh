#!/bin/bash
# Round-5 refresh on the closing tree: configs[2] (mixed objects, tag failures), file names,
# the host-resident (PCIe-inclusive) path, ranged 4 KiB reads (p50), and the self-launched
# 4-rank bench (gloo ranks sharing the box's GPU) with its configs[3] leg's digest.
set -o pipefail
OUT=gpurun_out/${1:-r05_cfg}
mkdir -p $OUT
timeout -k 10 300 python bench.py --mixed-gib 10 --no-cpu > $OUT/mixed.json 2> $OUT/mixed.err || { echo MIXED_FAILED; tail $OUT/mixed.err; exit 1; }
cut -c1-300 $OUT/mixed.json
RCLONE_AMD_NAME_TIMING=1 timeout -k 10 200 python bench.py --names 1000000 --no-cpu --steps 6 --warmup 2 > $OUT/names.json 2> $OUT/names.err || { echo NAMES_FAILED; tail $OUT/names.err; exit 1; }
cut -c1-200 $OUT/names.json
for b in 64 1024; do timeout -k 10 300 python tools/host_path_bench.py --batch $b >> $OUT/hostpath.json 2>>$OUT/hostpath.err || { echo HOSTPATH_FAILED; tail $OUT/hostpath.err; exit 1; }; done
cut -c1-300 $OUT/hostpath.json
for i in 1 2 3; do timeout -k 10 120 tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 >> $OUT/seek.jsonl 2>> $OUT/seek.err || { echo SEEK_FAILED; tail $OUT/seek.err; exit 1; }; done
cut -c1-300 $OUT/seek.jsonl
BENCH_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 4 --no-cpu > $OUT/bench4.json 2> $OUT/bench4.err || { echo BENCH4_FAILED; tail $OUT/bench4.err; exit 1; }
cut -c1-300 $OUT/bench4.json
echo CFG5_DONE
