# Round 4: config #3 at the reference's defaults (E=40 + early stopping, compaction on) under a kernel trace: where
# the sweep's wall time goes beyond the timed training kernels (idle gaps by the kernel that follows them, the
# untimed kernels: FedAvg, schedule, val / test evaluation, compaction copies).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04es_trace
rm -rf $O; mkdir -p $O
timeout -k 10 560 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --epochs 40 \
  --early-stopping --mnist-signal 0.2 --steps 1 --warmup 0 --no-cifar --no-shapley-agg --no-cpu-baseline \
  --budget-s 480 > $O/es.json 2> $O/es.err || { tail -5 $O/es.err; exit 12; }
python3 -c "
import json; d = json.loads(open('$O/es.json').read().strip().splitlines()[-1])
print('es', d['value'], d['ms_per_step'], json.dumps(d['early_stopping']))"
KSTATS_ROWS=30 KSTATS_W=60 python scripts/kstats.py $O/trace/run_kernel_stats.csv
python scripts/trace_gaps.py $O/trace/run_kernel_trace.csv 20
gzip $O/trace/run_kernel_trace.csv
