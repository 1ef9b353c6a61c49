set -o pipefail
mkdir -p gpurun_out
bash tools/e2e_r01_ab.sh 2>&1 | tee gpurun_out/e2eab.log
