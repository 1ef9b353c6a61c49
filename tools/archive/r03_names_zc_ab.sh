#!/bin/bash
# File names: the names GPU tests (zero-copy default), then bench.py --names with the name
# engine's zero-copy launch on vs off (XS_NAMES_ZERO_COPY), alternating.
set -o pipefail
OUT=gpurun_out/${1:-r03_names_zc}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_names_gpu.py > $OUT/names_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/names_tests.log; exit 1; }
tail -1 $OUT/names_tests.log
for i in 1 2 3; do for z in 1 0; do
  XS_NAMES_ZERO_COPY=$z timeout -k 10 200 python bench.py --names 1000000 --no-cpu --steps 20 --warmup 5 > $OUT/n.json 2> $OUT/n.err || { echo BENCH_FAILED; tail $OUT/n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/n.json')); print(json.dumps({'zero_copy': $z, 'names_per_s': d['value'], 'encrypt_s': d['encrypt_s'], 'decrypt_s': d['decrypt_s'], 'kernel': d.get('kernel')}))" | tee -a $OUT/names_ab.jsonl
done; done
