# HBM traffic of the dense kernels on the config #3 probe shape (252 coalitions x 5 partners, E=1):
# kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md HBM section).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_dense
rm -rf $O; mkdir -p $O
K='dense1_bwd_adam_kernel|dense_fwd_kernel'
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python scripts/probe_train.py 256 1 5 mnist > $O/trace.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python scripts/probe_train.py 256 1 5 mnist > $O/fetch.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python scripts/probe_train.py 256 1 5 mnist > $O/write.log 2>&1
rc=$?
echo EXIT $rc
exit $rc
