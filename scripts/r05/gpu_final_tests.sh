# Round 5 final check: the whole -m gpu suite on this tree (the reported count must match the code).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
[ $rc -eq 0 ] || exit $rc
# where config #2's 258 ms per sweep go: kernel trace of the Titanic leg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05lr -o run --output-format csv -- python bench.py --leg titanic --steps 3 --no-cpu-baseline > $O/titanic_trace.json 2> $O/titanic_trace.err && \
cp /tmp/r05lr/run_kernel_stats.csv $O/titanic_kernel_stats.csv
