# Round 5: kernel-trace stats of the driver's bench command on HEAD (the rocprof summary beside the bench line's
# in-stream kernel times) and the device-busy summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05trace
R=/tmp/r05trace
rm -rf $O $R; mkdir -p $O $R
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $R -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
cp $R/run_kernel_stats.csv $O/kernel_stats.csv
python scripts/trace_busy.py $R/run_kernel_trace.csv > $O/busy.txt 2>&1
head -12 $O/busy.txt
