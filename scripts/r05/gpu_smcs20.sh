# Round 5: the 20-partner SMCS GPU test alone (timed), then the Titanic kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_smcs20_gpu.py -m gpu -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider > $O/smcs20.log 2>&1 || { tail -30 $O/smcs20.log; exit 1; }
tail -4 $O/smcs20.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05lr -o run --output-format csv -- python bench.py --leg titanic --steps 3 --no-cpu-baseline > $O/titanic_trace.json 2> $O/titanic_trace.err && \
cp /tmp/r05lr/run_kernel_stats.csv $O/titanic_kernel_stats.csv && head -5 $O/titanic_kernel_stats.csv
