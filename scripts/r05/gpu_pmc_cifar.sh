# Round 5: HBM traffic of the config #4 leg's kernels: FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes of `bench.py --leg cifar` (no HIP events; every step's schedule stashed, so the line carries the
# algorithmic bytes of all launches), then scripts/pmc_traffic.py -> gpurun_out/r05pmc4/pmc_traffic_config4.json.
# Counters on the step's dominant kernel only (dense5_bwd, --kernel-include-regex): the first attempt, counters on
# every launch, aborted after ~40k dispatches with HSA_STATUS_ERROR_INVALID_PACKET_FORMAT inside the profiler's
# injected packets (profiles/r05_pmc_config4_fetch_failure.err); the same command without --pmc runs clean.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05pmc4
R=/tmp/r05pmc4
rm -rf $O $R; mkdir -p $O $R
CMD="python bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timer"
timeout -k 10 500 rocprofv3 --kernel-include-regex dense5_bwd_kernel --pmc FETCH_SIZE -d $R/fetch -o run --output-format csv -- $CMD > $O/fetch.json 2> $O/fetch.err && \
timeout -k 10 500 rocprofv3 --kernel-include-regex dense5_bwd_kernel --pmc WRITE_SIZE -d $R/write -o run --output-format csv -- $CMD > $O/write.json 2> $O/write.err
rc=$?
[ $rc -eq 0 ] && python scripts/pmc_traffic.py $R/fetch $R/write $O/fetch.json $O/pmc_traffic_config4.json > $O/pmc_traffic.txt 2>&1
echo "EXIT $rc"
tail -3 $O/fetch.err
exit $rc
