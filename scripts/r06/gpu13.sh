# Round 6: which change moved the MNIST numerics between the round-5 library and HEAD?  HEAD's host tree with
# (a) HEAD's library, (b) HEAD's library with the pre-refactor dense1_bwd_adam_kernel (gpurun_ab/oldd1.so); fusion off.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=distributed-learning-contributivity_amd/mplc/lib/libmplc_hip.so
cp $L gpurun_ab/keep.so
for v in keep oldd1; do
  cp gpurun_ab/$v.so $L
  MPLC_FUSE_AVG=0 timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_$v.log 2>&1
  echo "$v rc $? $(grep sha1 gpurun_out/hash_$v.log)"
done
cp gpurun_ab/keep.so $L
