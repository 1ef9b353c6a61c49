# configs[4] e2e at 32 GiB: round-1 build (tools/r01ab/, built from commit 1606c35) vs the current
# tree, alternating on one box.  Output: gpurun_out/e2eab_*.json
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for v in r01 cur; do
    exe=./tools/e2e_sync; [ $v = r01 ] && exe=./tools/r01ab/e2e_sync
    timeout -k 10 300 $exe --gib 32 --dir /dev/shm/e2eab_$$ --lanes 4 --transfers 16 > gpurun_out/e2eab_${v}_$i.json 2> gpurun_out/e2eab_${v}_$i.err
    rm -rf /dev/shm/e2eab_$$
    python3 -c "import json; d=json.loads(open('gpurun_out/e2eab_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', $i, d['sync_GiB_s'], d['cryptcheck_GiB_s'], d['lane_seconds'], d['ok'])"
  done
done
