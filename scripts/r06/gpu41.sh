# Round 6 final tree: every-rank emulation of config #3 (E=2) at N = 1, 2, 4, 8
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/emulate_ranks.py 2 0 0.0 1 2 4 8 > gpurun_out/r06_emulation_config3_e2.jsonl 2> gpurun_out/r06_emulation_config3_e2.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/r06_emulation_config3_e2.jsonl'):
    d = json.loads(l); print({k: d[k] for k in d if not isinstance(d[k], (list, dict))})"
