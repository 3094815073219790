set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/r06/gpu_ab_conv1.sh > gpurun_out/r06_ab_conv1.txt 2>&1 && \
bash scripts/r06/gpu_pmc_cifar.sh > gpurun_out/r06_pmc4.txt 2>&1
