#!/bin/bash
# configs[4] at full size (100 GiB) through the oracle-anchored GPU test; the harness JSON line is
# kept in gpurun_out/e2e_100.log.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
RCLONE_AMD_E2E_GIB=${E2E_GIB:-100} timeout -k 10 1120 python -u -m pytest -x -q -s --timeout 900 --timeout-method thread -p no:cacheprovider tests/test_e2e_anchor_gpu.py ${E2E_K:+-k $E2E_K} > gpurun_out/e2e_100.log 2>&1 || { echo E2E_FAILED; tail -30 gpurun_out/e2e_100.log; exit 1; }
grep -E "configs\[4\] e2e|^\{" gpurun_out/e2e_100.log | cut -c1-600
tail -1 gpurun_out/e2e_100.log
