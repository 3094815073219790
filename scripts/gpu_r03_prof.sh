# Round-3 profiles: config #4 leg's GPU busy fraction (kernel trace, no in-stream events), then the bench
# command's kernel-trace stats and the FETCH/WRITE passes (scripts/gpu_profile.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_cifar_busy.sh --no-kernel-timer && bash scripts/gpu_profile.sh ${1:-r03v1}
