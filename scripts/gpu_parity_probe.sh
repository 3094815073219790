set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
mkdir -p gpurun_out/parity
for v in wg8 wg9; do
  cp gpurun_ab/$v.so $L
  echo "== $v"
  timeout -k 10 400 python -u scripts/parity_probe.py > gpurun_out/parity/$v.log 2>&1 || { cp gpurun_ab/keep.so $L; tail -5 gpurun_out/parity/$v.log; exit 1; }
  tail -20 gpurun_out/parity/$v.log
done
cp gpurun_ab/keep.so $L
