# Round 6: the 10-partner ranking gate (tie band declared from the probe) and the rest of the -m gpu suite after
# test_shapley_gpu.py (the run before stopped at the 20-partner SMCS test: silent for > 180 s), with a heartbeat file
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
timeout -k 10 400 python -u -m pytest tests/test_ranking_gpu.py -m gpu -v -s --timeout 380 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06_ranking.log 2>&1
echo "ranking rc $?"
grep -E "device SV|v\(S\) mean|ranking:|PASSED|FAILED|Error" gpurun_out/r06_ranking.log | head -8
timeout -k 10 1000 python -u -m pytest tests/test_smcs20_gpu.py tests/test_variants_gpu.py tests/test_workload_gpu.py -m gpu -v \
  --timeout 600 --timeout-method thread --deselect tests/test_workload_gpu.py::test_config4_learned_accuracies_vs_oracle \
  -p no:cacheprovider > gpurun_out/r06_gpu_suite_rest.log 2>&1
rc=$?
kill $HB
grep -E "FAILED|passed|failed" gpurun_out/r06_gpu_suite_rest.log | tail -8
exit $rc
