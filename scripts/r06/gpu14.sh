# Round 6: Adam without contraction (every op rounded, Keras' order): model hash, then config #1's round-trajectory
# test and the MNIST / variant tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_adamoff.log 2>&1 || exit 1
grep sha1 gpurun_out/hash_adamoff.log
timeout -k 10 900 python -u -m pytest tests/test_config1_gpu.py tests/test_cnn_gpu.py tests/test_variants_gpu.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_adamoff_tests.log 2>&1
rc=$?
grep -o "((0, 2), 'W3', [0-9.e-]*, [0-9.e-]*)" gpurun_out/r06_adamoff_tests.log | head -1
tail -4 gpurun_out/r06_adamoff_tests.log
exit $rc
