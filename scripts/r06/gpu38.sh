# Round 6: host time between launches on the config #3 leg (the largest idle gaps of its kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
R=/tmp/gaps3; rm -rf $R
timeout -k 10 500 rocprofv3 --kernel-trace -d $R -o run --output-format csv -- python bench.py --leg train --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/gaps3.json 2> gpurun_out/gaps3.err || exit 1
python scripts/gaps_top.py $(find $R -name "*kernel_trace.csv" | head -1) 30 > gpurun_out/r06_gaps_config3.txt
python scripts/trace_busy.py $(find $R -name "*kernel_trace.csv" | head -1) | head -12 >> gpurun_out/r06_gaps_config3.txt
cat gpurun_out/r06_gaps_config3.txt
