# Round 5 final check: the whole -m gpu suite on this tree (the reported count must match the code).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05final
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
