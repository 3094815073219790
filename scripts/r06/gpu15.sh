# Round 6: the 10-partner ranking gate (fixture just made), then the full -m gpu suite on the round's kernels with
# -ffp-contract=on and contraction-free Adam (the config #4 E=2 gate waits for its fixture)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ranking_gpu.py -m gpu -v -s --timeout 380 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06_ranking.log 2>&1
echo "ranking rc $?"
grep -E "device SV|v\(S\) mean|PASSED|FAILED|Error" gpurun_out/r06_ranking.log | head -8
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  --deselect tests/test_ranking_gpu.py::test_ten_partner_exact_shapley_ranking_identical_to_oracle \
  --deselect tests/test_workload_gpu.py::test_config4_learned_accuracies_vs_oracle -p no:cacheprovider > gpurun_out/r06_gpu_suite.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r06_gpu_suite.log | tail -8
exit $rc
