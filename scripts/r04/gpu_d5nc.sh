# Round 4: (CIFAR) RMSprop updates without fused multiply-adds everywhere (#pragma clang fp contract(off) in
# rms_apply: the VALU dense5_bwd's SLP-packed mul + add never fused, the MFMA form's scalar code did) - rowenc = that
# change with the VALU dense5_bwd, d5mnc = with the MFMA dense5_bwd, expected bit-identical to each other;
# (MNIST) the MFMA dense1_bwd_adam with (d1m) and without (d1mnw) conv1's weights staged in LDS for
# conv_bwd_data / conv_wgrad; then the CIFAR / CNN / compaction GPU tests on the in-tree library (= d5mnc = d1mnw).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bad=0
V="rowe rowenc d5mnc rowe rowenc d5mnc" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|dense5|wino_kernel<13|total| v sha1"
[ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_rowenc/probe.log)" = "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_d5mnc/probe.log)" ] || { echo "HASH MISMATCH d5mnc"; bad=1; }
AB_VARIANTS="d1m d1mnw d1m d1mnw" bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_bwd_data|conv_wgrad|conv_fwd|dense1|total"
for v in d1m d1mnw; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
[ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_d1m/probe.log)" = "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_d1mnw/probe.log)" ] || { echo "MNIST HASH MISMATCH"; bad=1; }
timeout -k 10 900 python -u -m pytest tests/test_cifar_gpu.py tests/test_cnn_gpu.py tests/test_compaction_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -4 && [ $bad = 0 ]
