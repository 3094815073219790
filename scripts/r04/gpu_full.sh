# Round 4 checkpoint: the full -m gpu suite, then the driver's exact bench command (N=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_tests.sh > /dev/null 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/tests/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_driver_bench.sh > /dev/null 2>&1; rc=$?
cat gpurun_out/driver_bench/wall.txt
python3 -c "
import json; d = json.loads(open('gpurun_out/driver_bench/bench.json').read().strip().splitlines()[-1])
c4 = d.get('config4', {})
print('config3', d['value'], d['steps'], d['roofline']['frac'], 'config4', c4.get('value'), c4.get('config', {}).get('replicas_per_launch'))"
exit $rc
