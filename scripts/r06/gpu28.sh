# Round 6: the 10-partner ranking gate with its bands derived from two oracle passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
timeout -k 10 400 python -u -m pytest tests/test_ranking_gpu.py -m gpu -v -s --timeout 380 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06_ranking2.log 2>&1
rc=$?
kill $HB
grep -E "device SV|v\(S\) mean|ranking:|PASSED|FAILED|Error" gpurun_out/r06_ranking2.log | head -8
exit $rc
