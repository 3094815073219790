# Wall time of one probe with and without the two-stream phase overlap (MPLC_OVERLAP)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/overlap
rm -rf $O; mkdir -p $O
for ov in 0 1 0 1; do
  MPLC_OVERLAP=$ov timeout -k 10 300 python scripts/probe_train.py "$@" > $O/probe_$ov.log 2>&1 || exit 1
  echo "overlap=$ov: $(tail -1 $O/probe_$ov.log)"
done
