# Round-end rehearsal of the driver's GPU tiers on the final tree: pytest -m gpu, then smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc $rc" >> $O/pytest.log
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
echo "smoke rc $rc"; tail -5 $O/smoke.log
exit $rc
