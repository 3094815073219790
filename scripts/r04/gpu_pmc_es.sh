# Round 4: the CIFAR10 kernels' PMC passes (scripts/r04/gpu_pmc_cifar.sh), then config #3's E=40 + early-stopping
# sweep under a kernel trace (scripts/r04/gpu_es_trace.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/r04/gpu_pmc_cifar.sh > gpurun_out/r04_pmc_cifar.txt 2>&1 || { tail -20 gpurun_out/r04_pmc_cifar.txt; exit 21; }
tail -40 gpurun_out/r04_pmc_cifar.txt
bash scripts/r04/gpu_es_trace.sh
