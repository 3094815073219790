# Config #3 at the reference's defaults (E=40 + early stopping) with the val-evaluation time measured after a
# stream synchronisation; first the CIFAR10 round-trajectory test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03es2
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_workload_gpu.py::test_config4_round_trajectory_vs_fp64 -x -q -s \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python bench.py --epochs 40 --early-stopping --mnist-signal 0.2 --steps 1 --warmup 0 --no-cifar \
  --no-shapley-agg --no-cpu-baseline --budget-s 1100 > $O/es_bench.json 2> $O/es_bench.err || { tail -5 $O/es_bench.err; exit 12; }
python3 -c "
import json; d = json.loads(open('$O/es_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], json.dumps(d['early_stopping']))"
