#!/bin/bash
# Key-schedule field multiplies: column chains apart (XS_PMUL_SPLIT=1, the tree) vs carry-first (0):
# parity of every path that runs them, the fused phase marks, and the bulk keygen paired (abtest).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out/pmsplit
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py tests/test_ranged_open_gpu.py tests/test_gpu_parity.py tests/test_cipher_gpu.py \
  tests/test_engine_coalesce_gpu.py > gpurun_out/pmsplit/tests.log 2>&1 \
  || { echo TESTS_FAILED; tail -30 gpurun_out/pmsplit/tests.log; exit 1; }
tail -1 gpurun_out/pmsplit/tests.log
for i in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 60 ./tools/abtest_fp_pm$v 200 1 8 1 0x0006 > gpurun_out/pmsplit/probe_w0006_kg${v}_$i.json || { echo PROBE_FAILED; exit 1; }
    timeout -k 10 60 ./tools/abtest_fp_pm$v 200 1 8 1 > gpurun_out/pmsplit/probe_full_kg${v}_$i.json || { echo PROBE_FAILED; exit 1; }
  done
done
timeout -k 10 200 tools/abtest_pms 60 pms > gpurun_out/pmsplit/ab_pms.log 2>&1 || { echo AB_FAILED; exit 1; }
cat gpurun_out/pmsplit/ab_pms.log
echo pmsplit_done
