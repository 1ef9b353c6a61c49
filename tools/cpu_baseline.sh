#!/bin/bash
# GPU-box session: the drop-in's host paths with the GPU engine and with the CPU baseline engine
# (tests/native/cpu_engine.cpp, the vectorised oracle on host cores), back to back on one box:
#   * BASELINE configs[4] at E2E_GIB (default 100) GiB, both shapes: the batch shape (--lanes 4
#     --transfers 16) and rclone's per-object defaults (--transfers 4, --checkers 8), crypt.go:497-563;
#   * a ranged 4 KiB read (cipher.go:972-1034), 1 reader and 16 readers;
#   * with STREAM16=1 the per-object shape at --transfers 16 / --checkers 16 too (ONLY_STREAM16=1:
#     that alone).
# Output: gpurun_out/${1:-cpu_baseline}/*.json (one JSON line per run).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${1:-cpu_baseline}
GIB=${E2E_GIB:-100}
mkdir -p $OUT
make -s -C tests/native -j16 build/e2e_sync_cpu build/seek_latency_cpu > $OUT/make.log 2>&1 || { echo MAKE_FAILED; tail $OUT/make.log; exit 1; }
nproc > $OUT/host.txt; grep -m1 'model name' /proc/cpuinfo >> $OUT/host.txt; grep MemAvailable /proc/meminfo >> $OUT/host.txt
df -h /dev/shm >> $OUT/host.txt
TREE=/dev/shm/rc_e2e_cb_$$
run() {  # name, timeout, command...
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 $lim "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?
  rm -rf $TREE
  tail -c 600 $OUT/$name.json
  [ $rc -eq 0 ] || { echo "$name FAILED rc=$rc"; tail -5 $OUT/$name.err; exit 1; }
}
if [ -z "$ONLY_STREAM16" ]; then
run seek_gpu_t1 120 ./tools/seek_latency --mib 256 --reads 4000 --len 4096 --threads 1
run seek_cpu_t1 120 ./tests/native/build/seek_latency_cpu --mib 256 --reads 4000 --len 4096 --threads 1
run seek_gpu_t16 120 ./tools/seek_latency --mib 256 --reads 32000 --len 4096 --threads 16
run seek_cpu_t16 120 ./tests/native/build/seek_latency_cpu --mib 256 --reads 32000 --len 4096 --threads 16
run e2e_gpu_batch 900 ./tools/e2e_sync --gib $GIB --dir $TREE --lanes 4 --transfers 16
run e2e_cpu_batch 900 ./tests/native/build/e2e_sync_cpu --gib $GIB --dir $TREE --lanes 4 --transfers 16
run e2e_gpu_stream 900 ./tools/e2e_sync --gib $GIB --dir $TREE --mode stream --transfers 4 --check-mode stream --checkers 8
run e2e_cpu_stream 900 ./tests/native/build/e2e_sync_cpu --gib $GIB --dir $TREE --mode stream --transfers 4 --check-mode stream --checkers 8
fi
if [ -n "$STREAM16" ]; then  # the per-object shape at --transfers 16 / --checkers 16
run e2e_gpu_stream16 900 ./tools/e2e_sync --gib $GIB --dir $TREE --mode stream --transfers 16 --check-mode stream --checkers 16
run e2e_cpu_stream16 900 ./tests/native/build/e2e_sync_cpu --gib $GIB --dir $TREE --mode stream --transfers 16 --check-mode stream --checkers 16
fi
echo cpu_baseline_done
