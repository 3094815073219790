# Config #4 leg with the in-stream timer sampled per lockstep batch (bench.py CIFAR_TIMER_EVERY), then the
# round-3 profiles (scripts/gpu_r03_prof.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03cs
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u bench.py --leg cifar --steps 1 --warmup 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 31; }
python3 -c "
import json; c = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('config4', c['value'], c['ms_per_step'], c['roofline']['kernel'], c['roofline']['frac'], c['kernel_timer'])"
bash scripts/gpu_r03_prof.sh ${1:-r03v1}
