# Round 4 A/B round: CIFAR (xi-last Winograd weights, dense5_bwd row groups / staging chunk) on a config #4-shaped
# probe, then MNIST (conv_bwd_data un-pool without the compare / select chain) on the config #3-shaped probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/r04/gpu_ab_cifar.sh || exit 1
KSTATS_ROWS=8 KSTATS_W=40 AB_VARIANTS="cxil bwdup cxil bwdup" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_bwd|total"
for v in cxil bwdup; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
