# Round 6: config #4 counter passes over every launch, then the every-rank TMCS emulation with
# two HIP streams per rank, the CIFAR default now, at N = 1, 2, 4, 8.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/r06/gpu_pmc_cifar.sh > gpurun_out/r06_pmc4.txt 2>&1
rc=$?
echo "pmc rc $rc"
[ $rc -eq 0 ] || exit $rc
for n in 1 2 4 8; do
  timeout -k 10 400 python -u scripts/emulate_rank_mc.py $n > gpurun_out/r06_emulate_tmcs_n$n.txt 2> gpurun_out/r06_emulate_tmcs_n$n.err || exit 1
done
