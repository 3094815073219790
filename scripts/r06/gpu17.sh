# Round 6: the per-round reports of the two round-trajectory tests under the round's final numerics (Adam without
# contraction, -ffp-contract=on)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
MPLC_TRAJ_DUMP=gpurun_out/traj timeout -k 10 700 python -u -m pytest tests/test_workload_gpu.py tests/test_config1_gpu.py -m gpu -v -s \
  -k "round_trajectories" --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_traj.log 2>&1
rc=$?
kill $HB
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r06_traj.log | tail -5
exit $rc
