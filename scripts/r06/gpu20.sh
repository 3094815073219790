# Round 6: the GPU tests in test_contributivity.py / test_lr.py, then the driver's bench command on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_contributivity.py tests/test_lr.py -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06_gpu_suite_p3.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r06_gpu_suite_p3.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python bench.py > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err
rc=$?
tail -c 600 gpurun_out/r06_bench.json
exit $rc
