# Round profiles in one call: bench-command kernel trace + FETCH/WRITE passes (scripts/gpu_profile.sh <tag>),
# then the MFMA / wave-state PMC passes on the config #3 probe shape (scripts/gpu_pmc.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_profile.sh $1 && bash scripts/gpu_pmc.sh
