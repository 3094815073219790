# Round 5 emulation, third part: config #4 TMCS at N=8 with TMCS waves 4x and 16x (the product: world size, 8x).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05emu
mkdir -p $O
for w in 4 16; do
  timeout -k 10 400 python -u scripts/emulate_rank_mc.py 8 TMCS - $w > $O/c4_tmcs_n8_w$w.txt 2> $O/c4_tmcs_n8_w$w.err || exit 1
done
