# Round 4: config #3 at the reference's defaults (E=40 + early stopping) with early-stopping batch compaction, then
# an A/B of CIFAR dense5_bwd row groups per block (gpurun_ab/d5g{4,2,1}.so) on a config #4-shaped probe.
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
AB_VARIANTS="d5g4 d5g2 d5g1 d5g4" bash scripts/gpu_ab.sh 80 1 5 cifar 2>&1 | grep -E "==|dense5_bwd|sha1"
for v in d5g4 d5g2 d5g1; do grep -h sha1 gpurun_out/ab_$v/probe.log; done
