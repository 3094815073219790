# Round 4 final (part A): the whole -m gpu suite on the final library, then the driver's bench command (N=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r04final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04final/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04final/gpu_tests.log
[ $rc = 0 ] && bash scripts/gpu_driver_bench.sh
