# Round 4: dense5_fwd with 32 (and earlier 128 / 192) rows of W5 per K chunk (more loads in flight per chunk, half / a third of the
# barriers; the MFMA chain order is unchanged) against 64, on the CIFAR probe; bit-identity by v(S) hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bad=0
V="k64 k32 k64 k32" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|dense5|total| v sha1"
for v in k32; do [ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_k64/probe.log)" = "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)" ] || { echo "HASH MISMATCH $v"; bad=1; }; done
[ $bad = 0 ]
