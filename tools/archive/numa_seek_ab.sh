#!/bin/bash
# Ranged reads under NUMA placement on / off, 8 alternations (16 readers and 1 reader).
set -o pipefail
OUT=gpurun_out/${1:-numa_seek_ab}
mkdir -p $OUT
for i in 1 2 3 4 5 6 7 8; do
  for numa in 1 0; do
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 >> $OUT/seek16_$numa.jsonl &&
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 5000 --len 4096 --threads 1 >> $OUT/seek1_$numa.jsonl || { echo AB_FAILED; exit 1; }
  done
done
echo numa_seek_ab_done
