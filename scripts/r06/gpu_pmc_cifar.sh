# Round 6: the config #4 counter passes over EVERY launch, FETCH_SIZE and WRITE_SIZE in separate
# --pmc runs of `bench.py --leg cifar`, each with --kernel-trace (allowed beside --pmc) so that an abort names the
# dispatch it hit.  MPLC_CONCURRENT_BATCHES=1 reproduces round 5's failing run (one stream: the profiler serialises
# the dispatches anyway).  AMD_SERIALIZE_KERNEL=3 (the runtime waits on every kernel before and after it): with it
# the failing pass completes (scripts/r06/gpu_pmc4_diag.sh, profiles/r06_pmc4_diag_*), without it the pass aborts at
# the same batch in both rounds; counters are per dispatch, so serialising the host changes none of them.  The line carries every kernel's compulsory bytes of the same launches
# (algorithmic_bytes_per_launch_all.compulsory), set beside the counters by scripts/pmc_traffic.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06pmc4
R=/tmp/r06pmc4
rm -rf $O $R; mkdir -p $O $R
CMD="python bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timer"
MPLC_CONCURRENT_BATCHES=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/fetch -o run --output-format csv -- $CMD > $O/fetch.json 2> $O/fetch.err
rc=$?
echo "fetch rc $rc"
if [ $rc -ne 0 ]; then
  tail -40 $O/fetch.err
  for f in $(find $R/fetch -name "*kernel_trace.csv"); do wc -l $f; tail -5 $f > $O/fetch_trace_tail.csv; cp $f $O/ 2>/dev/null; done
  exit $rc
fi
MPLC_CONCURRENT_BATCHES=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/write -o run --output-format csv -- $CMD > $O/write.json 2> $O/write.err
rc=$?
echo "write rc $rc"
[ $rc -eq 0 ] && python scripts/pmc_traffic.py $R/fetch $R/write $O/fetch.json $O/pmc_traffic_config4.json > $O/pmc_traffic.txt 2>&1
tail -3 $O/fetch.err
exit $rc
