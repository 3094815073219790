# Round 4 final (part C): the driver's bench command on the final library (conv_fwd's per-wave loop off again), then
# config #4's SMCS at 20 partners once more on it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_driver_bench.sh && bash scripts/r04/gpu_smcs20.sh
