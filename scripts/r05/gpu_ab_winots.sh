# Round 5: CIFAR wino_kernel (conv3/conv4 forward and data gradients) with the T-plane tile stride CH + 4 (a
# half-wave's two tile quads on opposite bank halves) against HEAD's CH + 1, config #4-shaped probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=16 KSTATS_W=44 AB_VARIANTS="base cts base cts" timeout -k 10 900 bash scripts/gpu_ab.sh 52 1 5 cifar 2>&1 | grep -E "==|wino_kernel|total"
for v in base cts; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
