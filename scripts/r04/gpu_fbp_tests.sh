# Round 4: the CIFAR forward epilogues' bias loaded ahead (fbp: wave-local kernel in the last k-step, row form
# staged in LDS) against d5mnc (bit-identity by v(S) hash), then the whole -m gpu suite on the in-tree library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V="d5mnc fbp d5mnc fbp" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|wino|conv_kernel|total| v sha1"
[ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_d5mnc/probe.log)" = "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_fbp/probe.log)" ] || { echo "HASH MISMATCH fbp"; exit 32; }
mkdir -p gpurun_out/r04tests
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04tests/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r04tests/gpu_tests.log
exit $rc
