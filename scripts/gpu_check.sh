set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/probe_scale.py 64 5 400 > gpurun_out/probe_scale_small.log 2>&1 && \
timeout -k 10 400 python scripts/probe_scale.py 512 0 400 12 > gpurun_out/probe_scale.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then echo "probe rc $rc"; exit $rc; fi
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/pytest_gpu.log
echo EXIT $rc
