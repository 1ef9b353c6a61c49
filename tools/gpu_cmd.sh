set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/aql_launch 3000 tools/microbench/aql_kernel.co > gpurun_out/aql_launch.json 2> gpurun_out/aql_launch.err; rc=$?; cat gpurun_out/aql_launch.json; tail -5 gpurun_out/aql_launch.err; exit $rc
