# Round 5: LR kernel iteration (csrc/logreg.hip): parity tests, the phase timing copy, the Titanic leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05lr2
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lr.py tests/test_scenario.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/lr_tests.log 2>&1 || { tail -40 $O/lr_tests.log; exit 1; }
tail -3 $O/lr_tests.log
timeout -k 10 200 python scripts/lr_phases.py run $O/phases.json > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
python -c "import json; d=json.load(open('$O/phases.json')); print(d['newton_iterations'], d['fits'], {k: v['us_per_call'] for k, v in d['phases'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05lr2 -o run --output-format csv -- python bench.py --leg titanic --steps 5 --no-cpu-baseline > $O/titanic.json 2> $O/titanic.err || { tail -20 $O/titanic.err; exit 1; }
cp /tmp/r05lr2/run_kernel_stats.csv $O/titanic_kernel_stats.csv && head -3 $O/titanic_kernel_stats.csv && cut -c1-300 $O/titanic.json
