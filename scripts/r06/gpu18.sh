# Round 6: the full -m gpu suite on the round's final numerics, part 1 (test files up to test_shapley_gpu.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1100 python -u -m pytest $(ls tests/test_*gpu.py | grep -v -E "test_(smcs20|variants|workload|ranking)_gpu") -m gpu -v \
  --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_gpu_suite_p1.log 2>&1
rc=$?
kill $HB
grep -E "FAILED|passed|failed" gpurun_out/r06_gpu_suite_p1.log | tail -8
exit $rc
