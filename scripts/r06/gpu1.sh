set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/distributed-learning-contributivity_amd:$PWD/tests
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_concurrent_gpu.py > gpurun_out/r06_concurrent_tests.log 2>&1 && \
timeout -k 10 420 python -u scripts/probe_ranking.py --seeds 4 > gpurun_out/r06_probe_ranking.log 2>&1 && \
timeout -k 10 600 python -u scripts/diag_config3.py > gpurun_out/r06_diag_config3.log 2>&1
