#!/bin/bash
# Instruction-fetch stalls of the fused ranged-read kernel (tools/fused_probe, one block per launch,
# 4 KiB window): SQ wave-cycle counters in one pass, instruction-cache counters in another.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/icpmc
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY \
  --output-format csv -d gpurun_out/icpmc/a -o run -- ./tools/fused_probe 50 1 8 1 0x0006 > gpurun_out/icpmc/a.json || { echo PASS_A_FAILED; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES \
  --output-format csv -d gpurun_out/icpmc/b -o run -- ./tools/fused_probe 50 1 8 1 0x0006 > gpurun_out/icpmc/b.json || { echo PASS_B_FAILED; exit 1; }
find gpurun_out/icpmc -name "*counter_collection.csv" | head
echo icpmc_done
