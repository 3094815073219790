# Profiles of the bench command for the round's record: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (MI355X_MICROARCH.md HBM section) for the roofline kernels.  Raw rocprofv3 output stays
# under /tmp on the box (the bench command's trace is hundreds of MB); gpurun_out/profile_<tag> keeps the stats
# csv, the busy summary (scripts/trace_busy.py) and the per-launch traffic (scripts/pmc_traffic.py).
# bash scripts/gpu_profile.sh <tag> [pmc]   (pmc: the counter passes only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/profile_$1
R=/tmp/profile_$1
[ "$2" = pmc ] || rm -rf $O $R; mkdir -p $O $R
K='conv_bwd_data_kernel|conv_fwd_kernel|conv_wgrad_kernel|dense1_bwd_adam_kernel|dense1_bwd_adam_avg_kernel|dense_fwd_kernel|shapley_block_kernel'
CMD="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
# the counter passes run without the bench's in-stream HIP events (a --pmc pass with an event record around
# every launch crashed rocprofv3's counter thread: SIGSEGV, gpurun_out/profile_r02v6/fetch.err) and without
# the config #4, tutorial and Titanic sub-legs (their MNIST launches at other batch shapes would be averaged into
# the config #3 kernels' bytes per launch)
PMC="$CMD --no-kernel-timer --no-cifar --no-tutorial --no-titanic"
if [ "$2" != "pmc" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/trace -o run --output-format csv -- $CMD > $O/trace.json 2> $O/trace.err || exit $?
  cp $R/trace/run_kernel_stats.csv $O/kernel_stats.csv || exit 40
  python scripts/trace_busy.py $R/trace/run_kernel_trace.csv > $O/busy.txt 2>&1
  rm -rf $R/trace
fi
timeout -k 10 500 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE -d $R/fetch -o run --output-format csv -- $PMC > $O/fetch.json 2> $O/fetch.err && \
timeout -k 10 500 rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE -d $R/write -o run --output-format csv -- $PMC > $O/write.json 2> $O/write.err
rc=$?
[ $rc -eq 0 ] && python scripts/pmc_traffic.py $R/fetch $R/write $O/fetch.json $O/pmc_traffic.json > $O/pmc_traffic.txt 2>&1
echo "EXIT $rc"
du -sh $O
exit $rc
