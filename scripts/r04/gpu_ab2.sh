# Round 4 A/B: conv_bwd_data LDS-DMA form (MNIST probe), then dense5_bwd row groups (CIFAR probe).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/r04/gpu_ab_bwddma.sh || exit 1
V="cur cxg1 cxg2 cur cxg1" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|dense5_bwd|sha1| v sha1|total"
