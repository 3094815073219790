# Round 4: the driver's smoke() on the final library.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
