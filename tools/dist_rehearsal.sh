set -o pipefail
mkdir -p gpurun_out
export BENCH_DIST_BACKEND=gloo
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { echo FAIL2; tail -30 gpurun_out/dist2.err; exit 1; }
cat gpurun_out/dist2.json
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 2 --no-cpu > gpurun_out/dist4.json 2> gpurun_out/dist4.err || { echo FAIL4; tail -30 gpurun_out/dist4.err; exit 1; }
cat gpurun_out/dist4.json
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --object-blocks 400000 --no-cpu > gpurun_out/dist2_obj.json 2> gpurun_out/dist2_obj.err || { echo FAILOBJ; tail -30 gpurun_out/dist2_obj.err; exit 1; }
cat gpurun_out/dist2_obj.json
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29514 bench.py --gpus 2 --steps 2 --warmup 1 --names 200000 --no-cpu > gpurun_out/dist2_names.json 2> gpurun_out/dist2_names.err || { echo FAILNAMES; tail -30 gpurun_out/dist2_names.err; exit 1; }
cat gpurun_out/dist2_names.json
echo REHEARSAL_DONE
