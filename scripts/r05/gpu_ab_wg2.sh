# Round 5: CIFAR conv2 weight gradient with smaller bands (BTY 3 -> 2 / 1) and 3 waves per SIMD, against HEAD, on
# the config #4-shaped probe.  Kernel totals and the probe's v(S) hash (the tile order and the zero-padded k-step
# slots change, the per-output sums do not: bit-identical expected).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=20 KSTATS_W=44 AB_VARIANTS="base b2w3 b1w3 b2w2 base b2w3 b1w3 b2w2" timeout -k 10 1000 bash scripts/gpu_ab.sh 52 1 5 cifar 2>&1 | grep -E "==|wino_wgrad_kernel<32|total"
for v in base b2w3 b1w3 b2w2; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
