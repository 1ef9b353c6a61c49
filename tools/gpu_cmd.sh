set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r02g.e2e.jsonl
for ht in 0 8 0 8; do
  XS_MD5_HOST_THREADS=$ht timeout -k 10 300 ./tools/e2e_sync --gib 32 --dir /dev/shm/rc_e2e_ab --lanes 4 --transfers 16 >> gpurun_out/r02g.e2e.jsonl 2>>gpurun_out/r02g.e2e.err || { echo E2E_FAILED; tail gpurun_out/r02g.e2e.err; rm -rf /dev/shm/rc_e2e_ab; exit 1; }
  echo "host_threads=$ht done"
done
rm -rf /dev/shm/rc_e2e_ab
python3 -c "
import json
for l in open('gpurun_out/r02g.e2e.jsonl'):
    d=json.loads(l); print(d['sync_GiB_s'], d['cryptcheck_GiB_s'], d['lane_seconds'], d['ok'])
"
