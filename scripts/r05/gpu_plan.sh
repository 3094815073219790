# Round 5: config #4 TMCS with larger speculation budgets (mplc.mc.plan_frontier overhead 8 = default, 32, 128):
# replicas per lockstep batch vs coalitions trained, evals/s.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05plan
mkdir -p $O
for ov in 8 32 128; do
  timeout -k 10 300 python -u bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timer --mc-plan-overhead $ov > $O/ov$ov.json 2> $O/ov$ov.err || exit 1
  python -c "
import json; d=json.loads([l for l in open('$O/ov$ov.json') if l.startswith('{')][-1]); c=d['config']
print('overhead $ov:', d['value'], 'evals/s', c['coalitions_evaluated'], 'counted', c['coalitions_trained'], 'trained', round(c['replicas_per_launch']), 'replicas/launch', c['lockstep_batches'], 'batches', d['ms_per_step'], 'ms')"
done
