#!/bin/bash
# Wave key schedule in DPP rows (XS_KG_ROWS=1, the tree) vs 9-lane strides with LDS permutes (0):
# parity of every path that runs it, then the fused kernel's phase marks, alternating builds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out/kgrows
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py tests/test_ranged_open_gpu.py tests/test_gpu_parity.py tests/test_cipher_gpu.py \
  tests/test_engine_coalesce_gpu.py > gpurun_out/kgrows/tests.log 2>&1 \
  || { echo TESTS_FAILED; tail -30 gpurun_out/kgrows/tests.log; exit 1; }
tail -1 gpurun_out/kgrows/tests.log
for i in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 60 ./tools/abtest_fp_kg$v 200 1 8 1 0x0006 > gpurun_out/kgrows/probe_w0006_kg${v}_$i.json || { echo PROBE_FAILED; exit 1; }
    timeout -k 10 60 ./tools/abtest_fp_kg$v 200 1 8 1 > gpurun_out/kgrows/probe_full_kg${v}_$i.json || { echo PROBE_FAILED; exit 1; }
  done
done
echo kgrows_done
