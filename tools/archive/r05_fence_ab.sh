#!/bin/bash
# Round-5 A/B of the fused kernel's completion: one system-scope fence per
# workgroup (this tree) against one per wave (tools/microbench/ab_prev: the previous library, seek_latency_old
# linked to it with RUNPATH $ORIGIN; tools/microbench/launch_word_old built from the previous kernel
# file).  Parity tests of the fused / ranged / engine / shim paths and the fuzz first, then launch ->
# completion word (windowed and whole-block opens, host key setup, high-priority stream) and 4 KiB
# ranged reads through DecryptDataSeek (1 and 16 readers), alternating new / old; PROF_BOTH=1 adds a
# kernel trace of one 4 KiB run of each.  Also used for the even-split A/B (profiles/r05/even_split/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05_fence}
mkdir -p $OUT
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_fused_gpu.py tests/test_ranged_open_gpu.py tests/test_gpu_parity.py tests/test_cipher_gpu.py \
  tests/test_engine_coalesce_gpu.py tests/test_c_client_gpu.py tests/test_decrypter_fuzz_gpu.py > $OUT/tests.log 2>&1 \
  || { echo TESTS_FAILED; grep -E "FAILED|ERROR|Error" $OUT/tests.log | head -20; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
for i in $(seq ${PAIRS:-4}); do
  for v in new old; do
    if [ $v = old ]; then LW=tools/microbench/launch_word_old; SL=tools/microbench/ab_prev/seek_latency_old; else LW=tools/microbench/launch_word; SL=tools/seek_latency; fi
    for w in 0x2 0; do
      r=$(timeout -k 10 60 $LW 3000 1 2 $w) || { echo LW_FAILED $v; exit 1; }
      echo "{\"lib\": \"$v\", \"pair\": $i, \"launch_word\": $r}" >> $OUT/launch_word.jsonl
    done
    r=$(timeout -k 10 90 $SL --mib 256 --reads 5000 --len 4096 --threads 1) || { echo SEEK_FAILED $v; exit 1; }
    echo "{\"lib\": \"$v\", \"pair\": $i, \"seek\": $r}" >> $OUT/seek.jsonl
    r=$(timeout -k 10 90 $SL --mib 256 --reads 20000 --len 4096 --threads 16) || { echo SEEK16_FAILED $v; exit 1; }
    echo "{\"lib\": \"$v\", \"pair\": $i, \"seek\": $r}" >> $OUT/seek16.jsonl
  done
done
python3 - $OUT <<'PY'
import json, sys
d = sys.argv[1]
for l in open(d + "/launch_word.jsonl"):
    x = json.loads(l); r = x["launch_word"]
    print(x["lib"], "pair", x["pair"], "window", r["window"], "launch->word p50", r["launch_to_word_p50_us"], "p10", r["p10"], "p90", r["p90"])
for f in ("seek.jsonl", "seek16.jsonl"):
    for l in open(d + "/" + f):
        x = json.loads(l); r = x["seek"]
        print(f, x["lib"], "pair", x["pair"], "p50", r["p50_us"], "p90", r["p90_us"], "p99", r["p99_us"], "reads/s", r["reads_per_s"], "bad", r["bad"])
PY
if [ -n "$PROF_BOTH" ]; then export TMPDIR=/tmp; for v in new old; do if [ $v = old ]; then E=$R/tools/microbench/ab_prev/seek_latency_old; else E=$R/tools/seek_latency; fi; (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- $E --mib 256 --reads 2000 --len 4096 --threads 1 > $OUT/prof_$v.json 2>&1) || { echo PROF_FAILED $v; exit 1; }; done; for f in $(find $OUT/prof_new $OUT/prof_old -name "*kernel_stats.csv"); do echo "== $f"; python3 -c "import csv,sys; [print(r[\"Name\"][:50], r[\"Calls\"], round(float(r[\"AverageNs\"])/1000, 2), \"us\") for r in csv.DictReader(open(sys.argv[1])) if \"fused\" in r[\"Name\"]]" $f; done; fi
echo FENCE_AB_DONE
