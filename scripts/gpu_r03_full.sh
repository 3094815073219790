# Round 3 checkpoint: the whole -m gpu suite, smoke(), then the driver's bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03full
rm -rf $O; mkdir -p $O
timeout -k 10 840 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 31; }
tail -2 $O/smoke.log
timeout -k 10 620 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 32; }
python3 -c "
import json; d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('config3', d['value'], d['steps'], d['ms_per_step'], 'wall', d['wall_s_total']); print('roof', d['roofline']['kernel'], d['roofline']['frac'])
c = d['config4']; print('config4', c['value'], c['ms_per_step'], c['roofline']['kernel'], c['roofline']['frac'])
"
