# Round 4 final (part D): CIFAR / CNN GPU tests on the final library (dense5_fwd K chunk 32), then the bench command
# under a kernel trace with the FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_profile.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_cifar_gpu.py tests/test_cnn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 && \
bash scripts/gpu_profile.sh r04v5
