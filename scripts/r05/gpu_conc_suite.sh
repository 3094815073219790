# Round 5: CIFAR lockstep batches on two HIP streams by default: the concurrency test, the CIFAR / workload / variant
# GPU tests, then the config #4 bench leg (one TMCS run, its in-stream timer sampling 1 batch in 4, run in turn).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/conc; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_concurrent_gpu.py tests/test_cifar_gpu.py tests/test_variants_gpu.py tests/test_workload_gpu.py tests/test_planner.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline > $O/cifar.json 2> $O/cifar.err || { tail -5 $O/cifar.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/cifar.json').read().strip().splitlines()[-1])
print('config4', d['value'], d['ms_per_step'], d['roofline']['frac'] if d.get('roofline') else None)"
