# Round 5: CIFAR dense5_fwd in 16-sample x 64-column blocks on 16x16x4 MFMAs (d5n) against HEAD's 32 x 128 blocks on
# 32x32x2, on the config #4-shaped probe at 260 and 140 replicas (the per-rank batch at N=8).  Kernel totals and v(S)
# hashes (bit-identity expected).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for shape in "52 1 5 cifar" "28 1 5 cifar"; do
  echo "#### $shape"
  KSTATS_ROWS=24 KSTATS_W=44 AB_VARIANTS="base d5n base d5n" timeout -k 10 600 bash scripts/gpu_ab.sh $shape 2>&1 | grep -E "==|dense5_fwd|total" || exit 1
  for v in base d5n; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
done
