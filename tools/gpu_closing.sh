#!/bin/bash
# One GPU session on the current tree, in parts (gpurun's 1200 s limit):
#   A (default): the whole -m gpu suite (configs[4] at its full 100 GiB required:
#      RCLONE_AMD_E2E_REQUIRE_FULL=1, so a small box fails instead of skipping), smoke, the default
#      bench line (N = 1) and the self-launched 2-rank bench (gloo ranks sharing the GPU);
#   B (PROF=1): rocprofv3 kernel trace of the default bench command + timing agreement, then the
#      PMC passes (HBM bytes, VALU / MFMA counts) summarised per launch;
#   C (DIST=1): the multi-rank rehearsal (tools/dist_rehearsal.sh) including eight ranks (DIST8).
# usage: tools/gpu_closing.sh <tag>   (results under gpurun_out/<tag>/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-closing}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
export RCLONE_AMD_E2E_REQUIRE_FULL=1
if [ -z "$SKIP_A" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "PASSED|FAILED|ERROR" $OUT/gpu_tests.log | tail -20; tail -60 $OUT/gpu_tests.log; exit 1; }
grep -E "^configs\[(3|4)\]" $OUT/gpu_tests.log
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
fi
if [ -n "$BENCH2" ]; then
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --no-cpu > $OUT/bench2.json 2> $OUT/bench2.err || { echo BENCH2_FAILED; tail $OUT/bench2.err; exit 1; }
cut -c1-300 $OUT/bench2.json
fi
if [ -n "$PROF" ]; then
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -- python3 $R/bench.py --no-cpu > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail $OUT/prof.log; exit 1; }
cd $R && python3 tools/prof_agree.py $OUT/prof $OUT/prof.log $OUT/timing_agreement.json || echo prof_agree_failed
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc/p$i -- python3 $R/bench.py --no-cpu --no-pool-check --objectset-steps 0 --steps 10 > $OUT/pmc.p$i.log 2>&1 || { echo PMC_FAILED $i; tail -5 $OUT/pmc.p$i.log; exit 1; }
  i=$((i+1))
done
cd $R && python3 tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.json && echo PMC_DONE
fi
if [ -n "$DIST" ]; then
cd $R && DIST8=1 bash tools/dist_rehearsal.sh > $OUT/dist_rehearsal.log 2>&1 || { echo DIST_FAILED; tail -30 $OUT/dist_rehearsal.log; exit 1; }
cat $OUT/dist_rehearsal.log
for f in dist2 dist4 dist8 dist8_objset; do cp gpurun_out/$f.json $OUT/ 2>/dev/null; done
fi
echo CLOSING_DONE
