# Round 5 end: the driver's bench command on HEAD (the JSON line), then the kernel-trace stats of a short run of
# the same default leg (rocprof summary beside the line's in-stream kernel times) and the device-busy summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05end
R=/tmp/r05end
rm -rf $O $R; mkdir -p $O $R
timeout -k 10 590 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/trace.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
cp $R/run_kernel_stats.csv $O/kernel_stats.csv
python scripts/trace_busy.py $R/run_kernel_trace.csv > $O/busy.txt 2>&1
head -6 $O/busy.txt
