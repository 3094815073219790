# Round 6: the full -m gpu suite on the round's final numerics, part 2 (SMCS-20, variants, workload incl. the
# config #4 E=2 gate, the 10-partner ranking gate), then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1100 python -u -m pytest tests/test_smcs20_gpu.py tests/test_variants_gpu.py tests/test_workload_gpu.py \
  tests/test_ranking_gpu.py -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_final_suite_p2.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r06_final_suite_p2.log | tail -8
[ $rc -eq 0 ] && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_final_smoke2.log 2>&1
rc2=$?
kill $HB
cat gpurun_out/r06_final_smoke2.log | tail -3
[ $rc -eq 0 ] && exit $rc2
exit $rc
