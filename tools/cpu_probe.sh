#!/bin/bash
# Host CPU of the GPU box: model, vector extensions, CPU quota, and the MD5 rates per core
# (tools/microbench/md5_mb_rate: scalar vs 8 / 16 streams per core).
grep -m1 "model name" /proc/cpuinfo
grep -m1 flags /proc/cpuinfo | tr " " "\n" | grep -E "^(avx2|avx512f|avx512vl|avx512bw)$" | tr "\n" " "; echo
cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"
for i in 1 2 3; do ./tools/microbench/md5_mb_rate; done
