#!/bin/bash
# Paired A/B of NUMA placement (RCLONE_AMD_NUMA=1 vs 0), alternating, on the zero-copy host paths:
# 16 streams of 8 MiB and of 64 KiB objects (coalesce_bench) and 16 ranged readers (seek_latency).
set -o pipefail
OUT=gpurun_out/${1:-numa_ab}
mkdir -p $OUT
bash tools/numa_probe.sh > $OUT/probe.txt 2>&1
for i in 1 2 3 4; do
  for numa in 1 0; do
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/coalesce_bench 16 16 8388608 1 >> $OUT/cb8m_$numa.jsonl &&
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/coalesce_bench 16 800 65536 1 >> $OUT/cb64k_$numa.jsonl &&
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 >> $OUT/seek16_$numa.jsonl || { echo NUMA_AB_FAILED; exit 1; }
  done
done
echo numa_ab_done
