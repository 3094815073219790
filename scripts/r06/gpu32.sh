# Round 6 final tree: -m gpu suite part 1 (files up to test_shapley_gpu.py + test_contributivity / test_lr), smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest $(ls tests/test_*gpu.py | grep -v -E "test_(smcs20|variants|workload|ranking)_gpu") \
  tests/test_contributivity.py tests/test_lr.py -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06_final_suite_p1.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r06_final_suite_p1.log | tail -5
[ $rc -eq 0 ] && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_final_smoke.log 2>&1
rc2=$?
kill $HB
tail -2 gpurun_out/r06_final_smoke.log
[ $rc -eq 0 ] && exit $rc2
exit $rc
