# CIFAR probe A/B between the committed tree (gpurun_ab/oldtree: package + library as of HEAD) and the working
# tree: kernel trace of each and the v(S) hash.  bash scripts/gpu_ab_cifar.sh <probe args...>
# Prepare the old tree on the CPU side first:
#   git archive HEAD distributed-learning-contributivity_amd scripts/probe_train.py include | tar -x -C gpurun_ab/oldtree
#   (then build it there, or copy a library built from HEAD into its mplc/lib/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in old new old new; do
  O=gpurun_out/abc_$v; rm -rf $O; mkdir -p $O
  P=scripts/probe_train.py; [ $v = old ] && P=gpurun_ab/oldtree/scripts/probe_train.py
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python $P "$@" > $O/probe.log 2>&1 || exit 1
  echo "== $v"; python scripts/kstats.py $O/trace/run_kernel_stats.csv | head -14; grep sha1 $O/probe.log
done
