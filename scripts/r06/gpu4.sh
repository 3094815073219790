set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD:$PWD/distributed-learning-contributivity_amd:$PWD/tests
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cnn_gpu.py tests/test_concurrent_gpu.py > gpurun_out/r06_tests4.log 2>&1 && \
MPLC_FUSE_AVG=0 timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_fuse0.log 2>&1 && \
MPLC_FUSE_AVG=1 timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_fuse1.log 2>&1 && \
timeout -k 10 900 python -u scripts/probe_ranking.py --seeds 5 > gpurun_out/r06_probe_ranking4.log 2>&1
