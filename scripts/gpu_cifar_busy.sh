# GPU busy fraction of the config #4 leg (CIFAR10 TMCS, 20 partners): kernel trace summarised on the box
# (scripts/trace_busy.py), raw trace deleted.  bash scripts/gpu_cifar_busy.sh [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/cifar_busy
rm -rf $O; mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/cbtrace -o run --output-format csv -- python bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err
rc=$?
python scripts/trace_busy.py /tmp/cbtrace/run_kernel_trace.csv > $O/busy.txt 2>&1
cat $O/busy.txt | head -40
rm -rf /tmp/cbtrace
exit $rc
