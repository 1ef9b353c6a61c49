#!/bin/bash
# 32 per-object streams (16 GiB), 16-lane MD5 engine on / off, three alternations.
set -o pipefail
OUT=gpurun_out/${1:-r03_lanes32}
mkdir -p $OUT
D=/dev/shm/rc_e2e_l32
for i in 1 2 3; do
  for lanes in 1 0; do
    echo "lanes=$lanes" >> $OUT/cfg.txt
    XS_MD5_LANES=$lanes timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D --mode stream --check-mode stream --transfers 32 --checkers 32 >> $OUT/e2e16.jsonl 2>> $OUT/err.txt || { echo E2E_FAILED; rm -rf $D; exit 1; }
  done
done
rm -rf $D
python3 - $OUT <<'PY'
import json, sys
cfg = [l.strip() for l in open(sys.argv[1] + "/cfg.txt")]
for c, l in zip(cfg, open(sys.argv[1] + "/e2e16.jsonl")):
    r = json.loads(l); print(c, "sync", r["sync_GiB_s"], "check", r["cryptcheck_GiB_s"], "ok", r["ok"])
PY
