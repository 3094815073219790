# Round 5: MNIST conv_fwd's V rows as one fma by +-1 per value (fma1) instead of a multiply by +-1 and an fma (base),
# on the config #3-shaped probe (252 replicas): conv_fwd totals and v(S) hashes (bit-identity expected); then the
# MNIST CNN GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=6 KSTATS_W=40 AB_VARIANTS="base fma1 base fma1" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_fwd|total"
for v in base fma1; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py 2>&1 | tail -8
