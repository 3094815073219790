# Round 6 (VERDICT r5 missing 2 / item 4): the every-rank config #4 TMCS emulation with two HIP streams per rank (the
# CIFAR default now) at N = 1, 2, 4, 8 (round 5's one-stream numbers: profiles/r05_emulation_config4_tmcs.txt).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 1 2 4 8; do
  timeout -k 10 400 python -u scripts/emulate_rank_mc.py $n > gpurun_out/r06_emulate_tmcs_n$n.txt 2> gpurun_out/r06_emulate_tmcs_n$n.err || exit 1
  cat gpurun_out/r06_emulate_tmcs_n$n.txt
done
