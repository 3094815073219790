# Round 5 check 1: bit-identity of the pruned / pooled-stride CIFAR kernels and the split MNIST wgrad against the
# previous commit's tree (model rows hashed), then the new and changed GPU tests, then the Titanic bench leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c1
for w in ${HASH_MODELS-}; do
  timeout -k 10 300 python -u gpurun_ab/old_tree/scripts/model_hash.py $w 40 1 2>&1 | grep sha1 | sed "s/^/old /" || exit 1
  timeout -k 10 300 python -u scripts/model_hash.py $w 40 1 2>&1 | grep sha1 | sed "s/^/new /" || exit 1
done
timeout -k 10 1500 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_variants_gpu.py \
  tests/test_config1_gpu.py tests/test_cnn_gpu.py tests/test_cifar_gpu.py tests/test_lr.py -s > gpurun_out/r05c1/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r05c1/tests.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --leg titanic --steps 10 > gpurun_out/r05c1/titanic.json 2> gpurun_out/r05c1/titanic.err
tail -c 1500 gpurun_out/r05c1/titanic.json
