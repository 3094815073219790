# Round 6: (1) MNIST model hash of the pre-fusion tree (736103f + its library) and of HEAD on the SAME box - the
# recorded hashes moved between the two builds' calls (8276982736e43594 -> c3062b8960ee8a2c, fused or not);
# (2) config #1's round-trajectory test with the fused W3 average off and on.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
(cd gpurun_ab/t736 && timeout -k 10 300 python scripts/model_hash.py mnist 60 1) > gpurun_out/hash_t736.log 2>&1
echo "t736 rc $? $(grep sha1 gpurun_out/hash_t736.log)"
timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_head.log 2>&1
echo "head rc $? $(grep sha1 gpurun_out/hash_head.log)"
MPLC_FUSE_AVG=0 timeout -k 10 300 python scripts/model_hash.py mnist 60 1 > gpurun_out/hash_head0.log 2>&1
echo "head fuse0 rc $? $(grep sha1 gpurun_out/hash_head0.log)"
for f in 0 1; do
  MPLC_FUSE_AVG=$f timeout -k 10 300 python -u -m pytest tests/test_config1_gpu.py -m gpu -x -v --timeout 280 --timeout-method thread \
    -k "trajectories_vs_fp64" -p no:cacheprovider > gpurun_out/r06_traj_fuse$f.log 2>&1
  echo "traj fuse $f rc $?"
  grep -o "((0, 2), 'W3', [0-9.e-]*, [0-9.e-]*)" gpurun_out/r06_traj_fuse$f.log | head -1
done
