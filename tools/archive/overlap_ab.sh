# Engine submission A/B on one box, alternating three settings: "old" = shared condition with
# every waiter woken and no issue-while-waiting (XS_ENGINE_WAKE_ALL=1 XS_ENGINE_OVERLAP=0),
# "wake" = per-request wake-ups only (XS_ENGINE_OVERLAP=0), "new" = the defaults.  Ranged reads
# with 4 and 16 readers; 16 streaming handles of 64 KiB and 8 MiB objects.
# Output: gpurun_out/ov_<setting>.jsonl
set -e
cd $GRAFT_REPO_ROOT
run() {  # name, env...
  local n=$1; shift
  for t in 4 16; do
    env "$@" timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads $t >> gpurun_out/ov_$n.jsonl
  done
  env "$@" timeout -k 10 60 ./tools/coalesce_bench 16 800 65536 1 >> gpurun_out/ov_$n.jsonl
  env "$@" timeout -k 10 60 ./tools/coalesce_bench 16 16 8388608 1 >> gpurun_out/ov_$n.jsonl
}
for i in 1 2 3; do
  run old XS_ENGINE_WAKE_ALL=1 XS_ENGINE_OVERLAP=0
  run wake XS_ENGINE_OVERLAP=0
  run new XS_ENGINE_OVERLAP=1
done
echo overlap_ab_done
