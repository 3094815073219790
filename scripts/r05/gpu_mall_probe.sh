# Round 5: does the MI355X's memory-side cache help dense1_bwd_adam when a lockstep batch's W3 / Adam state
# (14 MB per replica) is small?  Kernel traces of the MNIST probe at 1260, 64, 32, 16 and 8 replicas; per-replica
# time of dense1_bwd_adam and dense_fwd.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05mall
rm -rf $O; mkdir -p $O
for cfg in "252 1 5" "32 1 2" "16 1 2" "8 1 2" "4 1 2"; do
  t=$(echo $cfg | tr ' ' _)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/mall_$t -o run --output-format csv -- python scripts/probe_train.py $cfg > $O/probe_$t.log 2>&1 || exit 1
  cp /tmp/mall_$t/run_kernel_stats.csv $O/stats_$t.csv
  echo "== $cfg"; grep -E "dense1_bwd_adam|dense_fwd" $O/stats_$t.csv | cut -d, -f1-4 | cut -c1-40,150-
done
