# Two-stream phase-interleave probe (scripts/probe_overlap.py): config #3's 1013 multi-partner coalitions
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03ov
rm -rf $O; mkdir -p $O
timeout -k 10 300 python scripts/probe_overlap.py 40 1013 single split lag single > $O/probe.log 2>&1
rc=$?
cat $O/probe.log | grep -v amdgpu.ids
exit $rc
