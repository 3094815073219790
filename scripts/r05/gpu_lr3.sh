# Round 5: the LR rounds as launches (fit work queue + averages): bitwise A/B against the one-wave-per-coalition
# build, the LR parity tests, the phase timing copy, the Titanic leg's kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05lr3
rm -rf $O; mkdir -p $O
timeout -k 10 300 python scripts/r05/lr_ab.py gpurun_ab/lr_old/libmplc_hip.so distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so $O > $O/ab.log 2>&1; rc=$?
tail -3 $O/ab.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_lr.py tests/test_scenario.py tests/test_native_sanitize.py tests/test_sbs.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/lr_tests.log 2>&1 || { tail -40 $O/lr_tests.log; exit 1; }
tail -3 $O/lr_tests.log
timeout -k 10 200 python scripts/lr_phases.py run $O/phases.json > $O/phases.log 2>&1 || { tail -20 $O/phases.log; exit 1; }
python -c "import json; d=json.load(open('$O/phases.json')); print(d['spans']['first_start_to_last_end_us'], {k: v['us_per_call'] for k, v in d['phases'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05lr3 -o run --output-format csv -- python bench.py --leg titanic --steps 5 --no-cpu-baseline > $O/titanic.json 2> $O/titanic.err || { tail -20 $O/titanic.err; exit 1; }
cp /tmp/r05lr3/run_kernel_stats.csv $O/titanic_kernel_stats.csv && head -6 $O/titanic_kernel_stats.csv | cut -c1-150 && cut -c1-300 $O/titanic.json
