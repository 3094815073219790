# Round 4 final (part B): config #3 at the reference's defaults (E=40 + early stopping, compaction on), then the bench
# command under a kernel trace with the FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_profile.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04es3
rm -rf $O; mkdir -p $O
timeout -k 10 500 python bench.py --epochs 40 --early-stopping --mnist-signal 0.2 --steps 1 --warmup 0 --no-cifar \
  --no-shapley-agg --no-cpu-baseline --budget-s 480 > $O/es.json 2> $O/es.err || { tail -5 $O/es.err; exit 33; }
python3 -c "
import json; d = json.loads(open('$O/es.json').read().strip().splitlines()[-1])
print('es', d['value'], d['ms_per_step'], json.dumps(d['early_stopping']))"
bash scripts/gpu_profile.sh r04v3
