# Round 4: config #4's SMCS at 20 partners, one whole run.  A CPU simulation on a real config #4
# v(S) table (scripts/sim_tmcs_planning.py) puts it at ~21.6k coalitions / ~216k replica-trainings (~750 s).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04smcs
rm -rf $O; mkdir -p $O
timeout -k 10 1120 python bench.py --leg cifar --method SMCS --cifar-partners 20 --steps 1 --warmup 0 --no-cpu-baseline \
  --budget-s 1100 > $O/smcs20.json 2> $O/smcs20.err || { tail -5 $O/smcs20.err; exit 13; }
python3 -c "
import json; d = json.loads(open('$O/smcs20.json').read().strip().splitlines()[-1])
print('smcs20', d['value'], d['ms_per_step'], d['config']['coalitions_evaluated'], d['config'].get('coalitions_trained'), d['config']['replicas_per_launch'], d['config']['lockstep_batches'])"
