# Round 6 final kernels: PMC summary of CIFAR conv1's forward (conv1_fwd_kernel, channels as the MFMA rows; round 5's
# conv_kernel<32,32,3,...> ran 12.6 VALU per MFMA) on the config #4-shaped probe, one stream, the runtime serialised
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
MPLC_CONCURRENT_BATCHES=1 AMD_SERIALIZE_KERNEL=3 bash scripts/gpu_pmc_probe.sh cifar_conv1 'conv1_fwd' 52 1 5 cifar > gpurun_out/r06_conv1_pmc.txt 2>&1 || { cat gpurun_out/r06_conv1_pmc.txt; exit 1; }
cat gpurun_out/r06_conv1_pmc.txt
