#!/bin/bash
# configs[4] at 100 GiB in the per-object shape at --transfers 16 / --checkers 16, anchored
# (the anchor records are checked against the CPU oracle afterwards, tools/check_anchor.py).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/e2e_s16
timeout -k 10 900 tools/e2e_sync --gib 100 --dir /dev/shm/rc_e2e_s16 --mode stream --transfers 16 --check-mode stream --checkers 16 --anchor gpurun_out/e2e_s16/anchor.jsonl > gpurun_out/e2e_s16/e2e.jsonl 2> gpurun_out/e2e_s16/e2e.err || { echo E2E_FAILED; tail gpurun_out/e2e_s16/e2e.err; rm -rf /dev/shm/rc_e2e_s16; exit 1; }
rm -rf /dev/shm/rc_e2e_s16
cut -c1-700 gpurun_out/e2e_s16/e2e.jsonl
