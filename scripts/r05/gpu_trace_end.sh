# Round 5 end: kernel-trace stats of a short run of the default bench leg on HEAD and the device-busy summary, with
# per-launch-grid averages (dense1_bwd_adam runs in the config #3 sweep and in the tutorial sub-leg at different
# batch shapes; the line's roofline is the config #3 launches').
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05end2
R=/tmp/r05end2
rm -rf $O $R; mkdir -p $O $R
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
cp $R/run_kernel_stats.csv $O/kernel_stats.csv
python scripts/trace_busy.py $R/run_kernel_trace.csv > $O/busy.txt 2>&1
head -3 $O/busy.txt; grep -A8 "by launch grid" $O/busy.txt
