# Monte-Carlo estimator legs (config #4 shape): TMCS at 20 partners, SMCS at 10 partners; per-batch replica
# counts in the line (config.replicas_per_launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/mc_bench
rm -rf $O; mkdir -p $O
timeout -k 10 400 python bench.py --leg cifar --method SMCS --cifar-partners 10 --warmup 0 --steps 1 --no-cpu-baseline --budget-s 380 > $O/smcs10.json 2> $O/smcs10.err && \
timeout -k 10 400 python bench.py --leg cifar --method TMCS --warmup 0 --steps 1 --no-cpu-baseline --budget-s 380 > $O/tmcs20.json 2> $O/tmcs20.err
rc=$?
for f in $O/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['coalitions_evaluated'], d['config']['replicas_per_launch'])"; done
exit $rc
