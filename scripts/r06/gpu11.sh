# Round 6: the full -m gpu suite on the round's kernels (the ranking and config #4 E=2 gates wait for their fixtures)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --deselect tests/test_ranking_gpu.py::test_ten_partner_exact_shapley_ranking_identical_to_oracle \
  --deselect tests/test_workload_gpu.py::test_config4_learned_accuracies_vs_oracle -p no:cacheprovider > gpurun_out/r06_gpu_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r06_gpu_suite.log
exit $rc
