# Round 4: config #3 at the reference's defaults (E=40 + early stopping) with early-stopping batch compaction (the
# default) and without (--compact-share 0), then config #4's SMCS at 20 partners.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04es
rm -rf $O; mkdir -p $O
timeout -k 10 500 python bench.py --epochs 40 --early-stopping --mnist-signal 0.2 --steps 1 --warmup 0 --no-cifar \
  --no-shapley-agg --no-cpu-baseline --budget-s 480 > $O/es_compact.json 2> $O/es_compact.err || { tail -5 $O/es_compact.err; exit 12; }
python3 -c "
import json; d = json.loads(open('$O/es_compact.json').read().strip().splitlines()[-1])
print('compact', d['value'], d['ms_per_step'], json.dumps(d['early_stopping']))"
timeout -k 10 600 python bench.py --leg cifar --method SMCS --cifar-partners 20 --steps 1 --warmup 0 --no-cpu-baseline \
  --budget-s 580 > $O/smcs20.json 2> $O/smcs20.err || { tail -5 $O/smcs20.err; exit 13; }
python3 -c "
import json; d = json.loads(open('$O/smcs20.json').read().strip().splitlines()[-1])
print('smcs20', d['value'], d['ms_per_step'], d['config']['coalitions_evaluated'], d['config']['replicas_per_launch'], d['config']['lockstep_batches'])"
