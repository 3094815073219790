# One-call GPU pass: GPU parity tests, smoke(), then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/round
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest_gpu.log
if [ $rc -ne 0 ]; then tail -40 $O/pytest_gpu.log; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/bench.json
echo EXIT $rc
