#!/bin/bash
# Round-5 A/B of the four-wave windowed-open kernel (xs_crypt_fused2<false, 4>)
# against the eight-wave kernel it replaces for ranged reads (XS_WINDOW_NCW=8), same library, same
# box: parity tests of the fused / ranged / engine / shim paths and the decrypter fuzz first, then
# launch -> completion word of one windowed open (tools/microbench/launch_word, host key setup,
# high-priority stream) and 4 KiB ranged reads through DecryptDataSeek (tools/seek_latency),
# alternating 8 / 4, then a kernel trace of one 4 KiB run of each.  Run with
# profiles/r05/window_4wave/win4_kernel.patch applied (not kept: it did not separate).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05_win4}
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
  for v in 8 4; do
    r=$(XS_WINDOW_NCW=$v timeout -k 10 60 tools/microbench/launch_word 3000 1 2 0x2) || { echo LW_FAILED $v; exit 1; }
    echo "{\"ncw\": $v, \"pair\": $i, \"launch_word\": $r}" >> $OUT/launch_word.jsonl
    r=$(XS_WINDOW_NCW=$v timeout -k 10 90 tools/seek_latency --mib 256 --reads 5000 --len 4096 --threads 1) || { echo SEEK_FAILED $v; exit 1; }
    echo "{\"ncw\": $v, \"pair\": $i, \"seek\": $r}" >> $OUT/seek.jsonl
    r=$(XS_WINDOW_NCW=$v timeout -k 10 90 tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16) || { echo SEEK16_FAILED $v; exit 1; }
    echo "{\"ncw\": $v, \"pair\": $i, \"seek\": $r}" >> $OUT/seek16.jsonl
  done
done
python3 - $OUT <<'PY'
import json, sys
d = sys.argv[1]
for l in open(d + "/launch_word.jsonl"):
    x = json.loads(l); r = x["launch_word"]
    print("ncw", x["ncw"], "pair", x["pair"], "launch->word p50", r["launch_to_word_p50_us"], "p10", r["p10"], "p90", r["p90"])
for f in ("seek.jsonl", "seek16.jsonl"):
    for l in open(d + "/" + f):
        x = json.loads(l); r = x["seek"]
        print(f, "ncw", x["ncw"], "pair", x["pair"], "p50", r["p50_us"], "p90", r["p90_us"], "reads/s", r["reads_per_s"], "bad", r["bad"])
PY
export TMPDIR=/tmp
for v in 8 4; do
  (cd /tmp && XS_WINDOW_NCW=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- $R/tools/seek_latency --mib 256 --reads 2000 --len 4096 --threads 1 > $OUT/prof_$v.json 2>&1) || { echo PROF_FAILED $v; exit 1; }
done
for f in $(find $OUT/prof_8 $OUT/prof_4 -name "*kernel_stats.csv"); do echo "== $f"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fused' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000, 2), 'us')" $f; done
echo WIN4_DONE
