# Kernel-trace profile of one probe run: bash scripts/gpu_probe.sh <out-name> <probe args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NAME=$1; shift
O=gpurun_out/probe_$NAME
rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python scripts/probe_train.py "$@" > $O/probe.log 2>&1
rc=$?
tail -3 $O/probe.log
python scripts/kstats.py $O/trace/run_kernel_stats.csv
exit $rc
