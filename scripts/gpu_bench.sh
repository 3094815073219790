# Round-end style measurement on one MI355X: bench line, kernel-trace stats of the same command,
# and FETCH_SIZE / WRITE_SIZE passes (separate, per the microarch guide) for the roofline `traffic`.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bench_r01
mkdir -p $O
K='conv_bwd_data_kernel|shapley_block_kernel'
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/trace.json 2> $O/trace.err && \
timeout -k 10 400 rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/fetch.json 2> $O/fetch.err && \
timeout -k 10 400 rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python bench.py --no-cpu-baseline > $O/write.json 2> $O/write.err
rc=$?
[ $rc -eq 0 ] && for n in 20 22 24 26; do
  timeout -k 10 120 python bench.py --leg shapley --n $n --no-cpu-baseline > $O/shapley_n$n.json 2>> $O/shapley.err || { rc=$?; break; }
done
echo EXIT $rc
