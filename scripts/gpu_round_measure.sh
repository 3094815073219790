# One call for the round's record: bench-command kernel trace + FETCH/WRITE passes (gpu_profile.sh <tag>), the
# driver's exact bench command (gpu_driver_bench.sh), then the config #3 rank emulation at 2/4/8 GPUs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_profile.sh $1 || exit $?
bash scripts/gpu_driver_bench.sh || exit $?
O=gpurun_out/emulate_$1
rm -rf $O; mkdir -p $O
for n in 2 4 8; do
  timeout -k 10 300 python scripts/emulate_rank.py $n >> $O/emulate.txt 2>> $O/emulate.err || exit $?
done
cat $O/emulate.txt
