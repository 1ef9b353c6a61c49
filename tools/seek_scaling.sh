#!/bin/bash
# Ranged 4 KiB reads vs reader count, GPU engine and CPU engine, plus the raw windowed-open
# scaling of the host cores (tests/native/par_open.cpp): where concurrent ranged reads stop scaling.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-seek_scaling}
mkdir -p $OUT
make -s -C tests/native -j16 build/seek_latency_cpu build/par_open > $OUT/make.log 2>&1 || { echo MAKE_FAILED; tail $OUT/make.log; exit 1; }
for t in 1 2 4 8 16; do
  timeout -k 5 60 ./tests/native/build/par_open $t 4000 >> $OUT/par_open.jsonl || exit 1
done
for t in 1 4 8 16; do
  timeout -k 5 120 ./tests/native/build/seek_latency_cpu --mib 256 --reads $((4000 * t)) --len 4096 --threads $t >> $OUT/seek_cpu.jsonl || exit 1
  timeout -k 5 120 ./tools/seek_latency --mib 256 --reads $((4000 * t)) --len 4096 --threads $t >> $OUT/seek_gpu.jsonl || exit 1
done
cat $OUT/par_open.jsonl
python3 -c "
import json
for f in ('seek_cpu', 'seek_gpu'):
    for l in open('$OUT/' + f + '.jsonl'):
        d = json.loads(l)
        print(f, d['threads'], 'p50', d['p50_us'], 'p99', d['p99_us'], 'reads/s', d['reads_per_s'], 'open/read/close us', d['mean_open_us'], d['mean_read_us'], d['mean_close_us'])
"
