# Round 6: do the HIP runtime's failed SDMA copies ("HSA copy failed with code 4097, falling to
# Blit copy", logged under the --pmc pass of scripts/r06/gpu_pmc4_diag.sh from the first batch of 534 replicas on)
# happen without the profiler?  The same config #4 leg, no rocprofv3, runtime errors logged (AMD_LOG_LEVEL=1).
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06copylog
rm -rf $O; mkdir -p $O
MPLC_CONCURRENT_BATCHES=1 AMD_LOG_LEVEL=1 timeout -k 10 200 python bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timer > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc $rc copy failures $(grep -c 'copy fail' $O/bench.err)"
exit $rc
