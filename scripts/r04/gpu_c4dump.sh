# Round 4, first GPU call: the CIFAR / ABI GPU tests on the ABI-2 library, then one config #4 TMCS run that
# dumps every trained v(S) (input of scripts/sim_tmcs_planning.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04c4
rm -rf $O; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_cifar_gpu.py tests/test_shapley_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline --dump-values $O/c4_values.npz > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/bench.err
exit $rc
