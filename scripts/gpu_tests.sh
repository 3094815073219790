# GPU parity tests of the given test files (default: all -m gpu), one process, per-test timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tests
rm -rf $O; mkdir -p $O
FILES=${@:-tests}
timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest.log
tail -40 $O/pytest.log
exit $rc
