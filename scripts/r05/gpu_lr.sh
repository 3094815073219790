# Round 5: the one-wave LR kernel (csrc/logreg.hip): the LR parity tests, the Titanic leg's kernel trace, then the
# config #4 PMC passes (scripts/r05/gpu_pmc_cifar.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05lr
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lr.py tests/test_scenario.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/lr_tests.log 2>&1 || { tail -40 $O/lr_tests.log; exit 1; }
tail -4 $O/lr_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05lr -o run --output-format csv -- python bench.py --leg titanic --steps 3 --no-cpu-baseline > $O/titanic_trace.json 2> $O/titanic_trace.err || { tail -20 $O/titanic_trace.err; exit 1; }
cp /tmp/r05lr/run_kernel_stats.csv $O/titanic_kernel_stats.csv && head -5 $O/titanic_kernel_stats.csv && cat $O/titanic_trace.json
bash scripts/r05/gpu_pmc_cifar.sh
