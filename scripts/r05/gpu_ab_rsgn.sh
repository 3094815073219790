# Round 5: CIFAR wino_kernel (conv3/conv4 forward and data gradients) with one fma by +-1 per V value and a single
# copy of the group loop (rsgn), against per-wave compiled copies with compile-time signs and the barriers inside
# the wave-divergent copies (base), on the config #4-shaped probe; kernel totals and v(S) hashes; then CIFAR tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=24 KSTATS_W=44 AB_VARIANTS="base rsgn base rsgn" timeout -k 10 600 bash scripts/gpu_ab.sh 52 1 5 cifar 2>&1 | grep -E "==|wino_kernel|total" || exit 1
for v in base rsgn; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cifar_gpu.py tests/test_variants_gpu.py 2>&1 | tail -3
