# Round 4: conv2's / conv4's gradients from the POOLED dz2 / dz4 (pdz2: dz2 only; pdz4: both) against the current
# library on the CIFAR probe: kernel trace and v(S) hash (bit-identity expected), then the CIFAR GPU tests on the
# in-tree library (= pdz4).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V="cur pdz2 pdz4 cur pdz4" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|dense5_bwd|wino_kernel<13|wino_wgrad_kernel<15, 15, 64, 64|wino_wl_kernel<30|wino_wgrad_kernel<32|wino_kernel<15, 15, 64, 32|total| v sha1"
a=$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_cur/probe.log)
for v in pdz2 pdz4; do b=$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log); [ "$a" = "$b" ] || { echo "HASH MISMATCH $v $a $b"; exit 2; }; done
timeout -k 10 600 python -u -m pytest tests/test_cifar_gpu.py tests/test_compaction_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
