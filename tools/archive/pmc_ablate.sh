#!/bin/bash
# PMC passes over a tools/ablate* binary (diagnostic builds of the crypt kernels).
# usage: tools/archive/pmc_ablate.sh <binary> <outdir-under-gpurun_out>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
BIN=$R/$1
OUT=$R/gpurun_out/$2
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -- $BIN > $OUT.p$i.log 2>&1
  i=$((i+1))
done
echo pmc_ablate_done
