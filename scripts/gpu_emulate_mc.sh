# Single-GPU emulation of rank 0 of an N-GPU config #4 TMCS run (scripts/emulate_rank_mc.py), N = 1, 2, 4, 8.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/emulate_mc
rm -rf $O; mkdir -p $O
rc=0
for n in 1 2 4 8; do
  timeout -k 10 420 python -u scripts/emulate_rank_mc.py $n TMCS >> $O/emulate.txt 2> $O/emulate_n$n.err || { rc=$?; break; }
done
cat $O/emulate.txt
exit $rc
