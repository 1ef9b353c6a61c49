#!/bin/bash
# Round 5 A/B, one box: configs[4] batch shape at 100 GiB with put checks inline, the library's
# host-MD5 routing of a group's longest objects on (default) vs off (XS_MD5_HOST_THREADS=0: every
# tee MD5 on the GPU lanes), alternating.  The host cores are the bound once the remote's MD5 runs
# inside each put, so routing work to them may cost more than it saves.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-r05_md5route}
mkdir -p $OUT
for i in 1 2; do
  for h in default 0; do
    if [ $h = default ]; then unset XS_MD5_HOST_THREADS; else export XS_MD5_HOST_THREADS=0; fi
    timeout -k 10 300 tools/e2e_sync --gib 100 --dir /dev/shm/rc_e2e_ab --lanes 4 --transfers 16 >> $OUT/e2e_$h.jsonl 2>> $OUT/e2e_$h.err || { echo E2E_FAILED; tail $OUT/e2e_$h.err; rm -rf /dev/shm/rc_e2e_ab; exit 1; }
    rm -rf /dev/shm/rc_e2e_ab
    tail -1 $OUT/e2e_$h.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('host_md5=$h', d['sync_GiB_s'], d['put_only_GiB_s'], d['cryptcheck_GiB_s'], d['ok'])"
  done
done
unset XS_MD5_HOST_THREADS
echo AB_DONE
