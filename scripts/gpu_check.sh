set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then echo "stop after pytest rc $rc"; exit $rc; fi
bash scripts/gpu_pmc.sh
