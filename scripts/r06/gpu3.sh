set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/distributed-learning-contributivity_amd:$PWD/tests
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lr.py::test_lr_evaluate_in_chunks_equals_one_call "tests/test_workload_gpu.py::test_config3_coalition_2_9_round_trajectories_vs_fp64" -s > gpurun_out/r06_tests3.log 2>&1 && \
timeout -k 10 1000 python -u scripts/probe_ranking.py --seeds 3 > gpurun_out/r06_probe_ranking3.log 2>&1
