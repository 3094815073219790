# Round 6: config #3 (the bench's train leg, one sweep, no kernel timer) on one HIP stream against two (each lockstep
# batch in two cost-balanced halves, MPLC_CONCURRENT_BATCHES=2), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r06_mnist_streams_leg.txt
for i in 1 2; do
  for c in 1 2; do
    MPLC_CONCURRENT_BATCHES=$c timeout -k 10 300 python bench.py --leg train --steps 1 --warmup 0 --no-kernel-timer \
      --no-cpu-baseline --no-cifar --no-titanic --no-tutorial --no-shapley-agg > gpurun_out/s$c.json 2> gpurun_out/s$c.err || exit 1
    python3 -c "
import json; d = json.loads(open('gpurun_out/s$c.json').read().strip().splitlines()[-1])
print('streams $c pass $i', d['value'], d['ms_per_step'], d['shapley_values'][:3])" | tee -a gpurun_out/r06_mnist_streams_leg.txt
  done
done
