# Full GPU pass: parity tests, smoke(), then the driver's exact bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_tests.sh && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/tests/smoke.log 2>&1 && \
bash scripts/gpu_driver_bench.sh
