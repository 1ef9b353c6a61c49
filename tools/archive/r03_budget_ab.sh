#!/bin/bash
# Per-object shapes at 32 and 64 streams (16 GiB): engines per device (RCLONE_AMD_DEVICES=0 vs
# 0,0,0,0), the 16-lane MD5 engine on / off, and the scalar-chain budget before lanes.
set -o pipefail
OUT=gpurun_out/${1:-r03_budget}
mkdir -p $OUT
D=/dev/shm/rc_e2e_b
run() { echo "$CFG" >> $OUT/cfg.txt; RCLONE_AMD_PHASES=1 timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D --mode stream --check-mode stream "$@" >> $OUT/e2e16.jsonl 2>> $OUT/phases.txt; }
for c in 64 32; do
  for devs in 0 0,0,0,0; do
    for cfg in "1 16" "0 16" "1 8"; do
      set -- $cfg
      CFG="c=$c devices=$devs lanes=$1 budget=$2" RCLONE_AMD_DEVICES=$devs XS_MD5_LANES=$1 XS_MD5_SCALAR_BUDGET=$2 run --transfers $c --checkers $c || { echo E2E_FAILED; tail $OUT/phases.txt; rm -rf $D; exit 1; }
    done
  done
done
rm -rf $D
python3 - $OUT <<'PY'
import json, sys
cfg = [l.strip() for l in open(sys.argv[1] + "/cfg.txt")]
rows = [json.loads(l) for l in open(sys.argv[1] + "/e2e16.jsonl")]
ph = [json.loads(l)["rclone_amd_phases"] for l in open(sys.argv[1] + "/phases.txt") if l.startswith("{")]
for c, r, p in zip(cfg, rows, ph):
    print(c, "| sync", r["sync_GiB_s"], "check", r["cryptcheck_GiB_s"], "ok", r["ok"], "| seal s enc/hash", round(p["enc_seal_s"]), round(p["hash_seal_s"]),
          "md5 wait", round(p["hash_md5_wait_s"]), "jobs w/i/l", p["md5_jobs_worker"], p["md5_jobs_inline"], p["md5_jobs_lanes"])
PY
