# Round 3: (1) the environment rocprofv3 --pmc gives the profiled program; (2) config #3 at the reference's
# defaults (E=40 + early stopping) once; (3) last, the one verification run of round 2's rocprofv3 --pmc
# crash: a FETCH_SIZE pass with the in-stream event timer forced on (MPLC_FORCE_KERNEL_TIMER), stderr kept.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03es
rm -rf $O; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES -d $O/envprobe -o envprobe -- python3 -c "import os; print({k: v for k, v in os.environ.items() if k.startswith('ROCP')})" > $O/env.txt 2>&1 || exit 11
grep -o "'ROCPROF_COUNTER[A-Z_]*': '[^']*'" $O/env.txt
timeout -k 10 1000 python bench.py --epochs 40 --early-stopping --mnist-signal 0.2 --steps 1 --warmup 0 --no-cifar \
  --no-shapley-agg --no-cpu-baseline --budget-s 1100 > $O/es_bench.json 2> $O/es_bench.err || exit 12
tail -c 900 $O/es_bench.json
MPLC_FORCE_KERNEL_TIMER=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o pmc -- python3 bench.py \
  --partners 5 --epochs 1 --steps 1 --warmup 0 --no-cifar --no-shapley-agg --no-cpu-baseline > $O/pmc_events.json 2> $O/pmc_events.err
rc=$?
echo "pmc-with-events rc=$rc"
tail -5 $O/pmc_events.err
exit 0
