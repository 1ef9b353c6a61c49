#!/bin/bash
# Round-5 A/Bs of the fused kernel: the VALU tag alone (profiles/r05/fused_vpoly/vpoly_kernel.patch)
# and the kept design (VALU tag for windowed opens + host key setup, profiles/r05/ranged_hybrid/).
# Fused small-batch kernel, VALU Poly1305 (this tree, with that patch applied) against the matrix-core tag (tools/ab_old/:
# the previous library and a seek_latency linked to it with RUNPATH $ORIGIN), on one box:
# parity tests of the fused / ranged / engine paths first, then ranged reads alternating
# new / old (4 KiB windowed reads and whole-block reads, one reader; 16 readers), then a
# kernel trace of one 4 KiB run of each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05_vpoly}
mkdir -p $OUT
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_fused_gpu.py tests/test_ranged_open_gpu.py tests/test_gpu_parity.py tests/test_extreme_gpu.py \
  tests/test_cipher_gpu.py tests/test_engine_coalesce_gpu.py tests/test_c_client_gpu.py > $OUT/tests.log 2>&1 \
  || { echo TESTS_FAILED; grep -E "FAILED|ERROR|Error" $OUT/tests.log | head -20; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
for i in $(seq ${PAIRS:-3}); do
  for v in new old; do
    if [ $v = old ]; then E=tools/ab_old/seek_latency_old; else E=tools/seek_latency; fi
    for cfg in "4096 1 2000" "65536 1 2000" "4096 16 20000"; do
      set -- $cfg
      r=$(timeout -k 10 90 $E --mib 256 --reads $3 --len $1 --threads $2) || { echo SEEK_FAILED $v $cfg; exit 1; }
      echo "{\"lib\": \"$v\", \"pair\": $i, \"result\": $r}" >> $OUT/seek.jsonl
    done
  done
done
python3 - $OUT/seek.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    print(d["lib"], d["pair"], "len", r["read_len"], "threads", r["threads"], "p50", r["p50_us"], "p90", r["p90_us"],
          "p99", r["p99_us"], "reads/s", r["reads_per_s"], "bad", r["bad"])
PY
export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then E=$R/tools/ab_old/seek_latency_old; else E=$R/tools/seek_latency; fi
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- $E --mib 256 --reads 2000 --len 4096 --threads 1 > $OUT/prof_$v.json 2>&1) || { echo PROF_FAILED $v; exit 1; }
done
for f in $(find $OUT/prof_new $OUT/prof_old -name "*kernel_stats.csv"); do echo "== $f"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fused' in r['Name'] or 'keygen' in r['Name'] or 'xs_open' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000, 2), 'us')" $f; done
echo VPOLY_DONE
