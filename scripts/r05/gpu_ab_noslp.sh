# Round 5: cifar_cnn.hip compiled with -fno-slp-vectorize and its two head kernels split into cifar_head.hip with
# the default flags (noslp: the product after the split) against the previous product (base), on the config
# #4-shaped probe at 260 replicas: kernel totals and v(S) hashes; then the CIFAR and variant GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for shape in "52 1 5 cifar"; do
  echo "#### $shape"
  KSTATS_ROWS=24 KSTATS_W=44 AB_VARIANTS="base noslp base noslp" timeout -k 10 600 bash scripts/gpu_ab.sh $shape 2>&1 | grep -E "==|wino|conv|dense|head|rmsprop|total" || exit 1
  for v in base noslp; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_variants_gpu.py tests/test_cifar_gpu.py 2>&1 | tail -18
