#!/bin/bash
# Per-object shapes at high concurrency (16 GiB): the 16-lane MD5 engine on (default) vs off
# (XS_MD5_LANES=0: every stream past the workers hashes on its own thread), alternating.
set -o pipefail
OUT=gpurun_out/${1:-r03_lanes}
mkdir -p $OUT
D=/dev/shm/rc_e2e_l
run() { RCLONE_AMD_PHASES=1 timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D --mode stream --check-mode stream "$@" >> $OUT/e2e16.jsonl 2>> $OUT/phases.txt; }
for c in 16 32 64; do
  for lanes in 1 0; do
    XS_MD5_LANES=$lanes run --transfers $c --checkers $c || { echo E2E_FAILED; tail $OUT/phases.txt; rm -rf $D; exit 1; }
  done
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
