# Round 6: MNIST on two HIP streams by default (as CIFAR10) and the bench's kernel timer on the first timed sweep only:
# -m gpu suite part 1 + smoke, then the driver's bench command (part 2 of the suite: scripts/r06/gpu33.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/r06/gpu32.sh || exit 1
bash scripts/r06/gpu40.sh || exit 1
