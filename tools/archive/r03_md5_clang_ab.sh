#!/bin/bash
# Host CPU of the box, and the scalar MD5 chain built by clang without / with the pinned add order
# (xs_host_md5.h XS_EARLY) next to the gcc build, 1 and 8 threads, alternating.
set -o pipefail
OUT=gpurun_out/${1:-r03_md5clang}
mkdir -p $OUT
grep -m1 "model name" /proc/cpuinfo > $OUT/cpu.txt
for i in 1 2; do
  for b in tools/ab_old/md5_clang_old tools/ab_old/md5_clang_new tools/microbench/md5_threads; do
    timeout -k 5 60 $b 1.5 1 8 | grep threads | sed "s#^{#{\"bin\": \"$(basename $b)\", #" >> $OUT/rates.jsonl || exit 1
  done
done
cat $OUT/cpu.txt $OUT/rates.jsonl
