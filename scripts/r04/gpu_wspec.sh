# Round 4: the conv kernels' main loops compiled once per wave (the wave's Winograd transform row makes the B^T / A
# signs compile-time: adds instead of multiplies by 0 / +-1).  CIFAR: wsp (wino_kernel + wino_wgrad_kernel) vs
# fbp; MNIST: mw (conv_wgrad) and mf (+ conv_fwd, 19 registers spilled) vs mb.  Bit-identity by v(S) hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bad=0
V="fbp wsp fbp wsp" bash scripts/r04/gpu_ab_cifar.sh 2>&1 | grep -E "==|wino|total| v sha1"
[ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_fbp/probe.log)" = "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_wsp/probe.log)" ] || { echo "HASH MISMATCH wsp"; bad=1; }
AB_VARIANTS="mb mw mf mb mw mf" bash scripts/gpu_ab.sh 252 1 5 2>&1 | grep -E "==|conv_bwd_data|conv_wgrad|conv_fwd|dense1|total"
for v in mb mw mf; do echo "$v $(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)"; done
for v in mw mf; do [ "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_mb/probe.log)" = "$(grep -ho 'v sha1 [0-9a-f]*' gpurun_out/ab_$v/probe.log)" ] || { echo "MNIST HASH MISMATCH $v"; bad=1; }; done
[ $bad = 0 ]
