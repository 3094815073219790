# Round 5: the config #4 TMCS leg with CIFAR lockstep batches on two persistent HIP streams (MPLC_CONCURRENT_BATCHES=2)
# against one stream, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/conc2; rm -rf $O; mkdir -p $O
for v in 2 1 2; do
  MPLC_CONCURRENT_BATCHES=$v timeout -k 10 300 python -u bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline > $O/c$v.json 2> $O/c$v.err || { tail -5 $O/c$v.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/c$v.json').read().strip().splitlines()[-1])
print('streams $v: config4', d['value'], d['ms_per_step'], d['roofline']['frac'] if d.get('roofline') else None, d['config']['shapley_estimate'][:3])"
done
