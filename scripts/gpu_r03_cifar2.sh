# CIFAR10 Winograd kernels: the all-kernel timer test, then config #4 (20-partner TMCS) with the per-kernel
# table; then the MNIST two-stream phase-overlap probe.  Each GPU step under its own time limit, chained.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03cifar2
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cifar_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "timer" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 21; }
tail -3 $O/pytest.log
timeout -k 10 400 python bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline --budget-s 380 > $O/cifar.json 2> $O/cifar.err || { tail -20 $O/cifar.err; exit 22; }
python3 -c "
import json; d = json.loads(open('$O/cifar.json').read().strip().splitlines()[-1])
print('config4', d['value'], 'evals/s', d['ms_per_step'], 'ms'); print('roofline', d['roofline'])
for k, e in d['kernels'].items(): print(k, e['ms_total'], e['time_share'], e.get('achieved'), e.get('frac'))
"
timeout -k 10 300 python scripts/probe_overlap.py 40 1013 single split lag single > $O/overlap.log 2>&1 || { tail -20 $O/overlap.log; exit 23; }
grep -v amdgpu.ids $O/overlap.log
