#!/bin/bash
# Phase times of the per-object shapes (RCLONE_AMD_PHASES=1), 16 GiB, workers 8 vs inline.
set -o pipefail
OUT=gpurun_out/${1:-r03_phases}
mkdir -p $OUT
D=/dev/shm/rc_e2e_p
for w in 8 0; do
  RCLONE_AMD_PHASES=1 XS_MD5_WORKERS=$w timeout -k 10 300 tools/e2e_sync --gib 16 --dir $D --mode stream --check-mode stream --transfers 4 --checkers 8 --check-dst-hash 0 >> $OUT/e2e.jsonl 2>> $OUT/phases_w$w.txt || { echo FAILED; tail $OUT/phases_w$w.txt; rm -rf $D; exit 1; }
done
rm -rf $D
cat $OUT/e2e.jsonl | cut -c1-400; tail -2 $OUT/phases_w*.txt
