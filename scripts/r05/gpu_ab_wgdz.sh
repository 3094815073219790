# Round 5: MNIST conv_wgrad with the windows' 2x2 delta staged un-pooled ([y00, y01, y10, y11] per channel, D by adds:
# dz4) against (value, argmax) pairs decoded per k-step (base), on the config #3-shaped probe: conv_wgrad totals and
# v(S) hashes (bit-identity expected); then the MNIST CNN GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KSTATS_ROWS=6 KSTATS_W=40 AB_VARIANTS="base dz4 base dz4" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_wgrad|total"
for v in base dz4; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cnn_gpu.py 2>&1 | tail -3
