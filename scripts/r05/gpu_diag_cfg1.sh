# Round 5: config #1 3-partner diagnosis (scripts/diag_config1.py) on the current library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/diag_config1.py > gpurun_out/diag_config1.log 2>&1
