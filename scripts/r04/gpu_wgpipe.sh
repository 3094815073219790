# Round 4: the CIFAR weight gradients' staging split into loads and LDS stores, the next band's loads in flight
# during this band's MFMAs (wgp1: conv2; wgp2: + conv4; wgp0: the split without the pipeline) against wsp.
# Bit-identity by v(S) hash; then the CIFAR GPU tests on the in-tree library (= wgp2).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bad=0
V="wsp wgp0 wgp1 wgp2 wsp wgp0 wgp1 wgp2" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|wgrad|total| v sha1"
for v in wgp0 wgp1 wgp2; do [ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_wsp/probe.log)" = "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)" ] || { echo "HASH MISMATCH $v"; bad=1; }; done
timeout -k 10 900 python -u -m pytest tests/test_cifar_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3 && [ $bad = 0 ]
