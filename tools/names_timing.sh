set -o pipefail
mkdir -p gpurun_out
RCLONE_AMD_NAME_TIMING=1 timeout -k 10 200 python bench.py --names 1000000 --no-cpu --steps 10 --warmup 3 > gpurun_out/nt.json 2> gpurun_out/nt.err || { echo FAIL; tail gpurun_out/nt.err; exit 1; }
tail -6 gpurun_out/nt.err; cat gpurun_out/nt.json | cut -c1-200
