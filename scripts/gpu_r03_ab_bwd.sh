# conv_bwd_data time split (timing-only variants, garbage gradients): staging / epilogue / MFMA compiled out
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_VARIANTS="${AB_VARIANTS:-bwd_base bwd_nostage bwd_noepi bwd_nomfma}" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5
