# Round 4: CIFAR row-kernel changes (rowx: XCD-aware block order for wino_kernel / dense5; rowe: + the data
# gradients' epilogue operand staged as bytes in LDS) against wlpm4 (ReLU' prefetch in the wave-local kernel), and
# the MNIST conv1 weights staged in LDS for conv_bwd_data's epilogue and conv_wgrad's recompute (mw1) against rowe;
# and dense1_bwd_adam on MFMA (d1m, bit-identical by construction); bit-identity by v(S) hash; then the CNN /
# CIFAR / compaction GPU tests on the in-tree library (= d5m: also dense5_bwd on MFMA, bit-identical by construction).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V="wlpm4 rowx rowe d5m wlpm4 rowx rowe d5m" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|wino|dense5|total| v sha1"
h=$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_wlpm4/probe.log)
bad=0
for v in rowx rowe d5m; do [ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)" = "$h" ] || { echo "HASH MISMATCH $v"; bad=1; }; done
AB_VARIANTS="rowe mw1 d1m rowe mw1 d1m" bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_bwd_data|conv_wgrad|conv_fwd|dense1|total"
for v in rowe mw1 d1m; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
for v in mw1 d1m; do [ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_rowe/probe.log)" = "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)" ] || { echo "MNIST HASH MISMATCH $v"; bad=1; }; done
timeout -k 10 900 python -u -m pytest tests/test_cifar_gpu.py tests/test_cnn_gpu.py tests/test_compaction_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -4 && [ $bad = 0 ]
