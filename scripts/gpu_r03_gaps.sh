# Idle time inside one config #3 sweep: kernel trace of the MNIST leg alone, gaps by neighbouring kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03gaps; rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/r03gaps -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cifar --no-shapley-agg --no-cpu-baseline --no-kernel-timer > $O/bench.json 2> $O/bench.err || exit 1
python scripts/gaps_context.py /tmp/r03gaps/run_kernel_trace.csv | tee $O/gaps.txt
python scripts/trace_busy.py /tmp/r03gaps/run_kernel_trace.csv > $O/busy.txt
