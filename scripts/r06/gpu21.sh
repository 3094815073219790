# Round 6: config #3's dense1 entry went 23.2 -> 25.5 ms per launch in the driver bench.  A/B on the config #3-shaped
# probe (252 coalitions, E=1): the pre-refactor dense1 kernel (oldd1: fusion on, Adam contracted), the refactor with
# Adam uncontracted (adamoff), the final build (cur: -ffp-contract=on), and cur with the fused W3 average off.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
KSTATS_ROWS=10 KSTATS_W=40 AB_VARIANTS="oldd1 adamoff cur oldd1 adamoff cur" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5 mnist > gpurun_out/r06_ab_dense1.txt 2>&1 || exit 1
O=gpurun_out/ab_fuse0; rm -rf $O; mkdir -p $O
MPLC_FUSE_AVG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python scripts/probe_train.py 252 1 5 mnist > $O/probe.log 2>&1 || exit 1
echo "== cur fuse0" >> gpurun_out/r06_ab_dense1.txt
KSTATS_ROWS=10 python scripts/kstats.py $O/trace/run_kernel_stats.csv >> gpurun_out/r06_ab_dense1.txt
grep -E "==|dense1|total" gpurun_out/r06_ab_dense1.txt
