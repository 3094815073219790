# Host-side (Python) profile of one emulated rank of an 8-GPU config #3 run: where the per-sweep fixed costs go.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/hostprof
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -m cProfile -o $O/prof.out scripts/emulate_rank.py 8 > $O/run.log 2>&1 || exit $?
cat $O/run.log | tail -2
python -c "
import pstats
p = pstats.Stats('$O/prof.out'); p.sort_stats('cumulative').print_stats(35)
" > $O/stats.txt 2>&1
head -80 $O/stats.txt
