# Round 5: multi-GPU emulation on the current kernels and planner: every rank's LPT shard
# trained alone for config #3 at E=2 (N=1,2,4,8), config #4 TMCS record-and-replay (N=2,4,8), and config #3 at
# E=40 + early stopping (N=1, 8).
set -o pipefail
export SKIP_E2=1
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05emu
mkdir -p $O
[ -n "$SKIP_E2" ] || { timeout -k 10 400 python -u scripts/emulate_ranks.py 2 0 0.0 1 2 4 8 > $O/c3_e2.jsonl 2> $O/c3_e2.err || exit 1; }
for n in 2 4 8; do
  timeout -k 10 400 python -u scripts/emulate_rank_mc.py $n TMCS > $O/c4_tmcs_n$n.txt 2> $O/c4_tmcs_n$n.err || exit 1
done
timeout -k 10 700 python -u scripts/emulate_ranks.py 40 1 0.2 8 1 > $O/c3_e40es.jsonl 2> $O/c3_e40es.err || exit 1
