# Round 6: where a small TMCS-sized CIFAR batch (25 coalitions x 5 partners = 125 replicas, what each rank trains per
# batch at N=8) spends its time: wall vs kernel busy (scripts/trace_busy.py), one and two streams
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 1 2; do
  O=gpurun_out/small_c$c; rm -rf $O; mkdir -p $O
  MPLC_CONCURRENT_BATCHES=$c timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python scripts/probe_train.py 25 1 5 cifar > $O/probe.log 2>&1 || exit 1
  python scripts/trace_busy.py $O/trace/run_kernel_trace.csv > $O/busy.txt 2>&1
  grep evals $O/probe.log; head -14 $O/busy.txt
  rm -rf $O/trace
done
for c in 1 2; do MPLC_CONCURRENT_BATCHES=$c timeout -k 10 300 python scripts/probe_train.py 25 1 5 cifar 2>&1 | grep evals | sed "s/^/plain c$c: /"; done
