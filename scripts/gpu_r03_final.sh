# Full -m gpu suite on the in-tree library, then the driver's exact bench command (N=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_tests.sh > /dev/null 2>&1; rc=$?
tail -3 gpurun_out/tests/pytest.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_driver_bench.sh > /dev/null 2>&1; rc=$?
cat gpurun_out/driver_bench/wall.txt
exit $rc
