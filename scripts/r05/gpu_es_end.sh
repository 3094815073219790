# Round 5 end: config #3 at the reference's defaults (E=40 + early stopping, learnable synthetic MNIST) on the final
# kernels: one whole sweep timed.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05es
rm -rf $O; mkdir -p $O
timeout -k 10 560 python bench.py --epochs 40 --early-stopping --mnist-signal 0.2 --steps 1 --warmup 0 --no-cifar \
  --no-titanic --no-tutorial --no-shapley-agg --no-cpu-baseline --budget-s 540 > $O/es.json 2> $O/es.err || { tail -5 $O/es.err; exit 12; }
python3 -c "
import json; d = json.loads(open('$O/es.json').read().strip().splitlines()[-1])
print('E40+ES', d['value'], d['ms_per_step'], json.dumps(d.get('early_stopping')))"
