set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ex_*.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_fused_gpu.py tests/test_engine_coalesce_gpu.py tests/test_readahead_gpu.py > gpurun_out/r02u.tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02u.tests.log; exit 1; }
tail -2 gpurun_out/r02u.tests.log
bash tools/express_ab.sh > gpurun_out/ex.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/ex.log; exit 1; }
python3 - <<'PY'
import json, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/ex_*.jsonl')):
    tag = f.split('ex_')[1].split('.')[0]
    for l in open(f):
        d = json.loads(l)
        if 'object_bytes' in d:
            agg[(tag, d['object_bytes'], d['readahead'])].append(d['GiB_s'])
        else:
            agg[(tag, 'seek16', 0)].append(d['reads_per_s'])
for k, v in sorted(agg.items(), key=str):
    print(k, v)
PY
