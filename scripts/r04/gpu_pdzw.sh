# Round 4: window-major un-pool staging (pdzw: each pooled value and code read once per window) against the round-3
# dense hand-off (cur) and the per-pixel un-pool (pdz4) on the CIFAR probe: kernel trace, v(S) hash (bit-identity
# expected), then the CIFAR GPU tests on the in-tree library (= pdzw).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V="cur pdz4 pdzw cur pdz4 pdzw" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|dense5_bwd|wino_kernel<13|wino_wgrad_kernel<15, 15, 64, 64|wino_wl_kernel<30|wino_wgrad_kernel<32|wino_kernel<15, 15, 64, 32|total| v sha1"
a=$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_cur/probe.log); b=$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_pdzw/probe.log)
[ "$a" = "$b" ] || { echo "HASH MISMATCH $a $b"; exit 2; }
timeout -k 10 600 python -u -m pytest tests/test_cifar_gpu.py tests/test_compaction_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
