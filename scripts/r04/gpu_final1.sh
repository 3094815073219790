# Round 4 measurement on the current library: the driver's bench command (N=1), then the bench command under a
# kernel trace and the FETCH_SIZE / WRITE_SIZE passes for the roofline kernels (scripts/gpu_profile.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_driver_bench.sh && bash scripts/gpu_profile.sh r04v2
