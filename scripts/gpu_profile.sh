# Profiles of the bench command for the round's record: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (MI355X_MICROARCH.md HBM section) for the roofline kernels.
# bash scripts/gpu_profile.sh <tag> [pmc]   (pmc: the counter passes only, into an existing <tag> directory)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/profile_$1
[ "$2" = pmc ] || rm -rf $O; mkdir -p $O
K='conv_bwd_data_kernel|conv_fwd_kernel|conv_wgrad_kernel|dense1_bwd_adam_kernel|dense_fwd_kernel|shapley_block_kernel'
CMD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
# the counter passes run without the bench's in-stream HIP events (a --pmc pass with an event record around
# every launch crashed rocprofv3's counter thread: SIGSEGV, gpurun_out/profile_r02v6/fetch.err)
PMC="$CMD --no-kernel-timer --no-cifar"
if [ "$2" != "pmc" ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $CMD > $O/trace.json 2> $O/trace.err || exit $?
fi
timeout -k 10 500 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $PMC > $O/fetch.json 2> $O/fetch.err && \
timeout -k 10 500 rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $PMC > $O/write.json 2> $O/write.err
rc=$?
echo "EXIT $rc"
exit $rc
