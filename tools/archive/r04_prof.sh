#!/bin/bash
# Round-4 measurement of the bench line's kernels: rocprofv3 kernel trace of the bench command
# (stats + HIP-event agreement) and the PMC passes for HBM traffic / VALU counts, stamped by
# tools/make_traffic.py into gpurun_out/<tag>/pmc_traffic.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04p}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -- python3 $R/bench.py --no-cpu > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail $OUT/prof.log; exit 1; }
cd $R && python3 tools/prof_agree.py $OUT/prof $OUT/prof.log $OUT/timing_agreement.json > /dev/null 2>&1 || echo prof_agree_failed
grep '^{' $OUT/prof.log | cut -c1-300
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc/p$i -- python3 $R/bench.py --no-cpu --steps 10 > $OUT/pmc.p$i.log 2>&1 || { echo PMC_FAILED $i; tail -5 $OUT/pmc.p$i.log; exit 1; }
  i=$((i+1))
done
cd $R && python3 tools/make_traffic.py $OUT/pmc $OUT/pmc_traffic.json > /dev/null && python3 tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.json && echo PMC_DONE
