#!/bin/bash
# Ranged-read work, round 3: parity of the keygen / fused paths, then ranged 4 KiB reads paired
# against the previous tree (tools/abprev, built in place), alternating, and the fused kernel's
# phase marks (tools/fused_probe).  Output under gpurun_out/rr_*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py tests/test_ranged_open_gpu.py tests/test_gpu_parity.py tests/test_engine_coalesce_gpu.py \
  tests/test_cipher_gpu.py tests/test_readahead_gpu.py > gpurun_out/rr_tests.log 2>&1 \
  || { echo TESTS_FAILED; tail -30 gpurun_out/rr_tests.log; exit 1; }
tail -1 gpurun_out/rr_tests.log
: > gpurun_out/rr_seek.jsonl
for i in 1 2 3; do
  for side in new old; do
    d=$R; [ $side = old ] && d=$R/tools/abprev
    timeout -k 10 60 $d/tools/seek_latency --mib 256 --reads 3000 --len 4096 --threads 1 > /tmp/s.json \
      || { echo SEEK_FAILED $side; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/s.json')); d['side']='$side'; d['run']=$i; print(json.dumps(d))" >> gpurun_out/rr_seek.jsonl
  done
done
python3 - <<'EOF'
import json
for l in open('gpurun_out/rr_seek.jsonl'):
    d = json.loads(l)
    print(d['side'], d['run'], {k: v for k, v in d.items() if 'p50' in k or 'p99' in k})
EOF
timeout -k 10 60 ./tools/fused_probe 200 1 8 1 > gpurun_out/rr_probe.json || { echo PROBE_FAILED; exit 1; }
timeout -k 10 60 ./tools/fused_probe 200 1 8 1 0x0006 > gpurun_out/rr_probe_w0006.json || { echo PROBE_FAILED; exit 1; }
timeout -k 10 60 ./tools/fused_probe 200 1 8 1 0x0001 > gpurun_out/rr_probe_w0001.json || { echo PROBE_FAILED; exit 1; }
timeout -k 10 60 ./tools/fused_probe 200 1 8 1 0x0400 > gpurun_out/rr_probe_w0400.json || { echo PROBE_FAILED; exit 1; }
echo rr_done
