# conv_bwd_data software-pipelined k-loop (BWD_PIPE, SLP off) vs the kept kernel: A/B kernel trace on the probe
# shape; the probe prints the v(S) hash (bit-identical results expected)
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_VARIANTS="${AB_VARIANTS:-new d1nc new d1nc}" timeout -k 10 900 bash scripts/gpu_ab.sh 252 1 5
for v in ${AB_VARIANTS:-new d1nc new d1nc}; do grep -o "evals/s.*sha1 [0-9a-f]*" gpurun_out/ab_$v/probe.log | sed "s/^/$v /"; done
