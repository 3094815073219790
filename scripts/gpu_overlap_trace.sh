# Kernel trace of the probe with the two-stream overlap on: do the halves' kernels run concurrently?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/overlap_trace
rm -rf $O; mkdir -p $O
MPLC_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python scripts/probe_train.py "$@" > $O/probe.log 2>&1
