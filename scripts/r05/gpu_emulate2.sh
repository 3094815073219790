# Round 5 emulation, second part: config #4 TMCS at N=4 / 8 with larger speculation budgets (mc_plan_overhead 32,
# 64 per rank), config #3 at E=40 + early stopping at N=1 (the N=8 shards: gpurun_out/r05emu/c3_e40es.jsonl).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05emu
mkdir -p $O
for a in "8 32" "8 64" "4 32"; do
  set -- $a
  timeout -k 10 400 python -u scripts/emulate_rank_mc.py $1 TMCS $2 > $O/c4_tmcs_n$1_ov$2.txt 2> $O/c4_tmcs_n$1_ov$2.err || exit 1
done
timeout -k 10 500 python -u scripts/emulate_ranks.py 40 1 0.2 1 > $O/c3_e40es_n1.jsonl 2> $O/c3_e40es_n1.err || exit 1
