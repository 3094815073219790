# Round 4: the new GPU tests (config #1 yml, multi-rank training, ES compaction) and the CIFAR / Shapley tests on
# the ABI-2 library, then one config #4 TMCS run with the speculative planner that dumps every trained v(S)
# (input of scripts/sim_tmcs_planning.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04c4
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_compaction_gpu.py tests/test_parallel_train_gpu.py tests/test_config1_gpu.py tests/test_cifar_gpu.py tests/test_shapley_gpu.py -m gpu -v -s --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -30
timeout -k 10 300 python -u bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline --dump-values $O/c4_values.npz > $O/bench.json 2> $O/bench.err
rc2=$?
tail -3 $O/bench.err
exit $(( rc != 0 ? rc : rc2 ))
