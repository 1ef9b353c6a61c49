#!/bin/bash
# Per-object shapes at 32 and 64 streams (16 GiB): how many scalar MD5 chains may run on host
# cores before streams go to the 16-lane engine (XS_MD5_SCALAR_BUDGET), and lanes off.
set -o pipefail
OUT=gpurun_out/${1:-r03_budget}
mkdir -p $OUT
D=/dev/shm/rc_e2e_b
run() { RCLONE_AMD_PHASES=1 timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D --mode stream --check-mode stream "$@" >> $OUT/e2e16.jsonl 2>> $OUT/phases.txt; }
for c in 32 64; do
  for b in 16 8 4 2; do
    XS_MD5_SCALAR_BUDGET=$b run --transfers $c --checkers $c || { echo E2E_FAILED; tail $OUT/phases.txt; rm -rf $D; exit 1; }
  done
  XS_MD5_LANES=0 run --transfers $c --checkers $c || { echo E2E_FAILED; rm -rf $D; exit 1; }
done
rm -rf $D
python3 - $OUT <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1] + "/e2e16.jsonl")]
ph = [json.loads(l)["rclone_amd_phases"] for l in open(sys.argv[1] + "/phases.txt") if l.startswith("{")]
for r, p in zip(rows, ph):
    print(r["transfers"], r["checkers"], "sync", r["sync_GiB_s"], "check", r["cryptcheck_GiB_s"], "ok", r["ok"],
          "jobs w/i/l", p["md5_jobs_worker"], p["md5_jobs_inline"], p["md5_jobs_lanes"])
PY
