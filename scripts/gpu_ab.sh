# A/B kernel-trace of one probe command with two prebuilt libraries: bash scripts/gpu_ab.sh <probe args...>
# (gpurun_ab/old.so and gpurun_ab/new.so, or the names in $AB_VARIANTS, built on the CPU side; the in-tree
# library is restored after).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in ${AB_VARIANTS:-old new}; do
  cp gpurun_ab/$v.so $L
  O=gpurun_out/ab_$v
  rm -rf $O; mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python scripts/probe_train.py "$@" > $O/probe.log 2>&1 || { cp gpurun_ab/keep.so $L; exit 1; }
  echo "== $v"; python scripts/kstats.py $O/trace/run_kernel_stats.csv
done
cp gpurun_ab/keep.so $L
