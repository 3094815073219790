# Round 6 final kernels: PMC summaries of the MNIST (config #3-shaped probe, 1260 replicas) and CIFAR10 (config #4-shaped
# probe, 260 replicas per launch, one stream, the runtime serialised as for every CIFAR counter pass this round) kernels
# - MFMA busy, VALU per MFMA, LDS bank-conflict ratio - for comparison with round 5's (profiles/r05_*_pmc_summary_end.txt)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_pmc_probe.sh mnist_r06 'conv_fwd|dense_fwd|dense1_bwd_adam_kernel|conv_bwd_data|conv_wgrad' 252 1 5 > gpurun_out/r06_mnist_pmc.txt 2>&1 || { cat gpurun_out/r06_mnist_pmc.txt; exit 1; }
cat gpurun_out/r06_mnist_pmc.txt
MPLC_CONCURRENT_BATCHES=1 AMD_SERIALIZE_KERNEL=3 bash scripts/gpu_pmc_cifar.sh > gpurun_out/r06_cifar_pmc.txt 2>&1 || { cat gpurun_out/r06_cifar_pmc.txt; exit 1; }
cat gpurun_out/r06_cifar_pmc.txt
