# Round 6 final tree: the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python bench.py > gpurun_out/r06_bench_last.json 2> gpurun_out/r06_bench_last.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r06_bench_last.json').read().strip().splitlines()[-1])
print('config3', d['value'], d['roofline']['frac'], json.dumps(d['kernels']['dense1_bwd_adam'].get('split')))
print('config4', d['config4']['value'], d['config4']['roofline']['frac'])"
