# Round 5: CIFAR conv4_fwd's 4-tile remainder group on v_mfma_f32_4x4x1f32 (quad = the product) against the padded
# 16-tile group (base, MPLC_WINO_QUAD=0) on the config #4-shaped probe at 260 replicas; kernel totals and v(S) hashes
# (bit-identity expected); then the variant-library test and the CIFAR GPU tests on the product library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for shape in "52 1 5 cifar"; do
  echo "#### $shape"
  KSTATS_ROWS=24 KSTATS_W=44 AB_VARIANTS="base quad base quad" timeout -k 10 600 bash scripts/gpu_ab.sh $shape 2>&1 | grep -E "==|conv4_fwd|wino_kernel|total" || exit 1
  for v in base quad; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_variants_gpu.py tests/test_cifar_gpu.py 2>&1 | tail -25
