#!/bin/bash
# round-3 measurement session: PMC passes on the current kernel sources (traffic + VALU/MFMA
# counters, stamped), the bench line with them, its rocprofv3 kernel trace, and a paired NUMA
# placement A/B (RCLONE_AMD_NUMA=0/1) of the zero-copy host paths.  Each GPU step has its own
# time limit; any failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${R03_TAG:-r03c}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
bash tools/pmc.sh ${T}_pmc --steps 5 --warmup 2 --no-cpu > $OUT/pmc.log 2>&1 || { echo PMC_FAILED; tail $OUT/pmc.log; ls $R/gpurun_out/; exit 1; }
cd $R
RCLONE_AMD_GIT_HEAD=${GIT_HEAD:-unknown} python3 tools/make_traffic.py gpurun_out/${T}_pmc $OUT/pmc_traffic.json > $OUT/make_traffic.log 2>&1 || { echo TRAFFIC_FAILED; cat $OUT/make_traffic.log; exit 1; }
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
python3 tools/pmc_summary.py gpurun_out/${T}_pmc > $OUT/pmc_summary.json
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -- python3 $R/bench.py --no-cpu > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail $OUT/prof.log; exit 1; }
cd $R
python3 tools/prof_agree.py $OUT/prof $OUT/prof.log $OUT/timing_agreement.json > /dev/null 2>&1 || echo prof_agree_failed
for i in 1 2; do
  for numa in 1 0; do
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/coalesce_bench 16 16 8388608 1 >> $OUT/numa_cb8m_$numa.jsonl &&
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/coalesce_bench 16 800 65536 1 >> $OUT/numa_cb64k_$numa.jsonl &&
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 1 >> $OUT/numa_seek1_$numa.jsonl &&
    RCLONE_AMD_NUMA=$numa timeout -k 10 60 ./tools/seek_latency --mib 256 --reads 20000 --len 4096 --threads 16 >> $OUT/numa_seek16_$numa.jsonl || { echo NUMA_AB_FAILED; exit 1; }
  done
done
python3 -c "import ctypes; L=ctypes.CDLL('rclone_amd/librclone_crypt.so'); print('device0_numa_node', L.xs_device_numa_node(0))" > $OUT/numa_node.txt
echo MEASURE_DONE
