# Round 6: what runs in the last seconds of config #3's timed step (host gaps between small torch kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
R=/tmp/gaps3b; rm -rf $R
timeout -k 10 300 rocprofv3 --kernel-trace -d $R -o run --output-format csv -- python bench.py --leg train --steps 1 --warmup 0 \
  --no-cpu-baseline --no-cifar --no-titanic --no-tutorial --no-shapley-agg > gpurun_out/gaps3b.json 2> gpurun_out/gaps3b.err || exit 1
T=$(find $R -name "*kernel_trace.csv" | head -1)
python scripts/gaps_top.py $T 20 > gpurun_out/r06_gaps_config3_only.txt
python scripts/kernels_window.py $T 0 0.3 > gpurun_out/r06_kernels_head.txt
L=$(python scripts/kernels_window.py $T 0 0 | tail -1 | awk '{print $5}')
python scripts/kernels_window.py $T $(python3 -c "print($L - 3.0)") $L > gpurun_out/r06_kernels_tail.txt
head -25 gpurun_out/r06_gaps_config3_only.txt; grep -v "gap     0.0" gpurun_out/r06_kernels_tail.txt | awk '$3 > 1.0' | head -60
