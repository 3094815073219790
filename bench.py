"""Benchmark driver (contract: one JSON line on rank 0).

python bench.py [--gpus N] [--steps K] [--warmup W] [--leg train|shapley|cifar|titanic] [--budget-s B]

leg "train" (default; BASELINE.json metric "coalition v(S) evals/sec (MNIST FedAvg)"): BASELINE config #3
  - MNIST CNN, 10 partners, random split ([0.1]*10), FedAvg, exact "Shapley values" over all 1023
  coalitions, M=20 minibatches, G=8 gradient updates per pass, fixed E=2 epochs (no early stopping, so
  the work is deterministic).  MNIST-shaped synthetic data (x ~ U[0,1) fp32
  [60000,28,28,1], random one-hot labels; no network for the dataset), resident in HBM before timing.
  One step = one full Contributivity.compute_contributivity("Shapley values"): train + test-evaluate all
  1023 coalitions (batched, lockstep), then the exact-Shapley aggregation.  value = coalitions / second.
  Multi-GPU: coalitions LPT-sharded over ranks, v(S) assembled by one RCCL all_reduce (strong scaling:
  the job is fixed).
  Also reported: "shapley_agg" - the exact-Shapley aggregation kernel on a 2^28 fp64 table (config #5).
leg "shapley": only the N=28 aggregation (GB/s).
leg "titanic" (BASELINE config #2): Titanic-shaped data, 10 partners, FedAvg logistic regression (E=3, M=1), exact
  "Shapley values" over all 1023 coalitions; value = coalitions / second.  Also the "config2" sub-object of the
  default line, beside the oracle's single-thread rate and the reference's own measured 10.1 evals/s.
leg "cifar" (BASELINE config #4): CIFAR10 CNN, 20 partners, FedAvg, "TMCS" (default; --method SMCS etc.) with
  the reference's defaults (sv_accuracy .01, alpha .95, truncation .05), fixed E=1, M=20, G=8.  CIFAR10-shaped
  synthetic data with class templates (signal 0.4: accuracy grows with the data a coalition holds, so the
  truncation behaves as on real data; CIFAR10 itself cannot be fetched).  One step = one full
  compute_contributivity(method) with numpy seeded 0; value = distinct coalitions evaluated / second.

Wall-clock budget.  One training step is a whole contributivity computation (about 40 s for config #3 on one
MI355X), so the driver's `--steps 20 --warmup 5` would not fit its 600 s limit.  The run is held to
--budget-s seconds from process start (default 480, covering interpreter start, warm-up, the timed steps,
the N=28 aggregation leg and the CPU baseline): warm-up is capped at one step (it only pays the one-time
allocation of the lockstep batch), and the timed region runs the largest K' <= K whole steps that the
measured warm-up step says will fit.  The line reports K' as "steps" (and the requested K as
"steps_requested"); every timed step is complete, nothing inside a step is skipped.  A heartbeat goes to
stderr after every step.
"""
import argparse
import json
import os
import sys
import time

T_PROC0 = time.perf_counter()  # before `import torch` (its first import on a fresh box can take minutes)

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "distributed-learning-contributivity_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X fp32 matrix peak (v_mfma_f32_32x32x2_f32), spec
# conv2's data gradient per sample.  The kernel runs it in Winograd form F(2x2,3x3): 169 output tiles x 16
# transform points x 64 x 32 multiply-adds, all fp32 - that algorithm's arithmetic is the roofline count.  The
# direct convolution (every conv1 position x 32 x 576) is 2.25x more and is reported beside it only as the
# equivalent rate: priced against the MFMA peak it would read as ~100 % while the matrix cores are half idle.
CONV_BWD_DATA_FLOP_PER_SAMPLE = 169 * 16 * 64 * 32 * 2
CONV_BWD_DATA_DIRECT_FLOP_PER_SAMPLE = 676 * 32 * 576 * 2
MNIST_FWD_FLOP = 23984896       # per sample, SURVEY A21
MNIST_TRAIN_FLOP = 71565312     # per sample (fwd + wgrad + dgrad, no conv1 dgrad)
# The training step's kernels (csrc/mnist_cnn.hip, timed in stream with HIP events) and the algorithmic unit of
# each: (bound, unit of the rate, units per sample or the stash key, description).  The convolutions are priced at
# the Winograd F(2x2,3x3) algorithm's own conv2 multiply-adds (what the matrix cores execute); the W3 kernels at
# the HBM bytes their access pattern must move.
WINO_FWD_FLOP_PER_SAMPLE = 144 * 16 * 32 * 64 * 2  # 144 pool-window tiles x 16 points x 32 ci x 64 co
KERNEL_UNITS = {
    "conv_fwd": ("mfma", "TFLOP/s", WINO_FWD_FLOP_PER_SAMPLE,
                 "conv2's Winograd multiply-adds, 144 tiles x 16 points x 32 x 64 per sample"),
    "dense_fwd": ("hbm", "GB/s", "dense_fwd_bytes", "W3 read + the pooled row read and hidden row written per sample"),
    "head": (None, None, None, "Dense(10) + softmax-CE + Adam(W4): one block per replica, latency-bound"),
    "dense1_bwd_adam": ("hbm", "GB/s", "dense1_bwd_adam_bytes",
                        "W3 read and written, Adam moments read/written by optimizer step, pooled + dh read and "
                        "dpooled written per sample"),
    "conv_bwd_data": ("mfma", "TFLOP/s", CONV_BWD_DATA_FLOP_PER_SAMPLE,
                      "the data gradient's Winograd multiply-adds, 169 tiles x 16 points x 64 x 32 per sample"),
    "conv_wgrad": ("mfma", "TFLOP/s", WINO_FWD_FLOP_PER_SAMPLE,
                   "dW2's Winograd F(3x3,2x2) multiply-adds, 144 tiles x 16 points x 32 x 64 per sample"),
    "adam_small": (None, None, None, "Adam on W1/b1/W2/b2 from the per-sample partials"),
}
TRAIN_KERNELS = list(KERNEL_UNITS)


def kernel_table(timer, units):
    """Per training kernel: launches, in-stream ms (HIP events on the launch stream), share of the step's kernel
    time and, for the kernels with an algorithmic unit, the achieved rate against its roofline."""
    tot = sum(timer.total_ms(k) for k in TRAIN_KERNELS) or 1.0
    out = {}
    for k, (bound, unit, per, desc) in KERNEL_UNITS.items():
        ms, n = timer.total_ms(k), timer.launches(k)
        e = {"launches": n, "ms_total": round(ms, 1), "ms_avg": round(ms / max(1, n), 4),
             "time_share": round(ms / tot, 4)}
        if bound is not None and ms > 0 and units:
            amount = units[per] if isinstance(per, str) else units["samples"] * per
            if bound == "hbm":
                rate, peak = amount / (ms / 1000) / 1e9, HBM_PEAK_GBS
            else:
                rate, peak = amount / (ms / 1000) / 1e12, FP32_MFMA_PEAK_TFLOPS
            e.update({"bound": bound, "achieved": round(rate, 2), "peak": peak, "unit": unit,
                      "frac": round(rate / peak, 4), "units_per_launch": int(amount / max(1, n)), "algorithmic": desc})
        out[k] = e
    return out


def dense1_split(eng, timer):
    """The dense1_bwd_adam entry over its two kinds of step (ABI 4): the steps without the fused W3 average (one
    dense pass per replica) and a FedAvg round's last step (dense1_bwd_adam_kernel for the replicas outside fused
    coalitions + dense1_bwd_adam_avg_kernel, timed between the same two events).  Per launch ms from the in-stream
    timer in step order, beside each step's own algorithmic bytes (MnistModel.algorithmic_units of its stash
    record)."""
    ms = timer.per.get("dense1_bwd_adam", [])
    recs = timer.stash
    if not ms or len(ms) != len(recs):
        return None
    acc = {"unfused_steps": [0, 0.0, 0.0], "fused_steps": [0, 0.0, 0.0]}
    for t, rec in zip(ms, recs):
        fused = len(rec) > 3 and bool((rec[3] > 0).any().item())
        e = acc["fused_steps" if fused else "unfused_steps"]
        e[0] += 1
        e[1] += t
        e[2] += eng.model_impl.algorithmic_units([rec])["dense1_bwd_adam_bytes"]
    out = {}
    for k, (n, t, b) in acc.items():
        if n:
            rate = b / (t / 1000) / 1e9
            out[k] = {"launches": n, "ms_avg": round(t / n, 4), "achieved": round(rate, 2), "unit": "GB/s",
                      "frac": round(rate / HBM_PEAK_GBS, 4), "bytes_per_launch": int(b / n)}
    out["note"] = ("a FedAvg round's last step runs the fused W3 average (dense1_bwd_adam_avg_kernel: each block walks "
                   "its coalition's replicas in turn) in place of the replicas' W3 stores and the aggregation's W3 "
                   "reads; the entry above covers both kinds of step")
    return out


TRAFFIC_SOURCE = ("profiles/pmc_traffic.json: FETCH_SIZE / WRITE_SIZE from separate rocprofv3 --pmc passes of "
                  "this same command (scripts/pmc_traffic.py), not measured in this run")


def log(msg):
    print(f"[bench {time.perf_counter() - T_PROC0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def host_threads():
    """Host CPU threads this process may use.  On the GPU box OMP_NUM_THREADS carries the job's CPU share
    (16 per GPU) while os.cpu_count() reports every core of the shared host, so the smaller one is used."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


PMC_FILES = ("pmc_traffic.json", "pmc_traffic_config4.json")  # config #3 (+ #5), config #4


def pmc_entry(kernel, workload):
    """The committed PMC record of `kernel` for the bench command of `workload` (profiles/pmc_traffic*.json, written
    by scripts/pmc_traffic.py): bytes per launch, and for config #4 the algorithmic bytes of the same launches."""
    for name in PMC_FILES:
        try:
            with open(os.path.join(REPO, "profiles", name)) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        if doc.get("workload") == workload and kernel in doc.get("kernels", {}):
            return doc["kernels"][kernel]
    return None


def pmc_by_launch(name, workload):
    """config #4: the counters' bytes of launch `name` (mplc.cifar.launch_name: conv2_fwd, dense5_bwd, ...) over
    every launch of the profiled run beside its compulsory bytes (profiles/pmc_traffic_config4.json by_launch)."""
    for fname in PMC_FILES:
        try:
            with open(os.path.join(REPO, "profiles", fname)) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        if doc.get("workload") == workload and name in doc.get("by_launch", {}):
            return doc["by_launch"][name]
    return None


# launches timed as one entry of the kernel table: a round's last MNIST step runs dense1_bwd_adam_kernel for the
# unfused replicas and dense1_bwd_adam_avg_kernel for the fused coalitions between the same two events (ABI 4)
PMC_FOLD = {"dense1_bwd_adam_kernel": ("dense1_bwd_adam_avg_kernel",)}


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the committed PMC passes of this same bench command (the launches folded
    into its timing entry, PMC_FOLD, added in); None when absent or for another workload."""
    e = pmc_entry(kernel, workload)
    if e is None:
        return None
    total, n = float(e["traffic_bytes_per_launch"]) * e["launches"], e["launches"]
    for k in PMC_FOLD.get(kernel, ()):
        f = pmc_entry(k, workload)
        if f is not None:
            total += float(f["traffic_bytes_per_launch"]) * f["launches"]
    return int(total / max(1, n))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv=None):
    """`python bench.py --gpus N` without an outer launcher: start N ranks of this same command as child
    processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, one GPU each) and return the
    exit status.  The parent never touches the GPU (no torch.cuda call: it only starts and watches the
    children), so nothing here replaces a process that initialised the device.  Rank 0 prints the JSON line
    (its stdout is this process's stdout).  When a rank fails, the others are stopped: they would otherwise
    wait in a collective for the dead one."""
    import signal
    import subprocess
    argv = [os.path.abspath(__file__)] + sys.argv[1:] if argv is None else list(argv)
    port = _free_port()
    procs = []

    def forward(signum, frame):  # the parent is stopped (driver time limit, ^C): take the ranks with it
        for q in procs:
            if q.poll() is None:
                os.killpg(q.pid, signal.SIGKILL if signum != signal.SIGINT else signal.SIGTERM)
        sys.exit(128 + signum)
    for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(sig, forward)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MPLC_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, "-u"] + argv, env=env, start_new_session=True,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    log(f"launched {n} ranks (pids {[p.pid for p in procs]}, master 127.0.0.1:{port})")
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log(f"rank {procs.index(p)} exited with {code}: stopping the other ranks")
                for q in live:
                    os.killpg(q.pid, signal.SIGTERM)
        time.sleep(0.2)
    for q in procs:
        q.wait()
    return rc


def dist_init(expected=None, use_gpu=True):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if expected is not None and world != expected:
        raise SystemExit(f"bench.py: --gpus {expected} but the launcher started WORLD_SIZE={world} ranks")
    if not use_gpu:
        if world > 1 and not dist.is_initialized():
            dist.init_process_group("gloo")
        return int(os.environ.get("RANK", "0")), world, None
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; more ranks than GPUs (a gloo rehearsal of the multi-rank path on a 1-GPU box)
    # share them round-robin
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    backend = os.environ.get("MPLC_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI; gloo for rehearsals
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    return rank, world, dev


def barrier(world):
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world):
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def run_budgeted(warm_step, timed_step, args, world, reserve_s, what, max_steps=None, warmup=None):
    """Warm-up (at most one step of `warm_step`) + timed steps of `timed_step(i, planned)` under the wall-clock
    budget.  Returns (steps run, warm-up steps run, wall seconds of the timed region (max over ranks), the last
    step's result, per-step seconds).  Every rank takes the same decisions: they are made from max-over-ranks
    times."""
    warm = min(args.warmup if warmup is None else warmup, 1)
    t_step = 0.0
    for _ in range(warm):
        t = time.perf_counter()
        warm_step()
        barrier(world)
        t_step = max_over_ranks(time.perf_counter() - t, world)
        log(f"{what}: warm-up step {t_step:.1f}s")
    elapsed = max_over_ranks(time.perf_counter() - T_PROC0, world)
    left = args.budget_s - elapsed - reserve_s
    steps = args.steps if max_steps is None else min(args.steps, max_steps)
    requested = steps
    if t_step > 0:
        steps = max(1, min(steps, int(left // (t_step * 1.03))))
    log(f"{what}: timing {steps} of {requested} requested steps ({left:.0f}s left for them)")
    barrier(world)
    t0 = time.perf_counter()
    res = None
    done = 0
    per_step = []
    for i in range(steps):
        ts = time.perf_counter()
        res = timed_step(i, steps)
        done += 1
        per_step.append(time.perf_counter() - ts)
        log(f"{what}: step {i + 1}/{steps} {per_step[-1]:.1f}s")
        if t_step == 0 and done < steps:
            # no warm-up estimate: stop early rather than overrun (decided on rank-0's clock, broadcast by max)
            over = (time.perf_counter() - T_PROC0) + (time.perf_counter() - ts) + reserve_s > args.budget_s
            if max_over_ranks(1.0 if over else 0.0, world) > 0:
                break
    barrier(world)
    wall = max_over_ranks(time.perf_counter() - t0, world)
    per_step = [max_over_ranks(t, world) for t in per_step]
    return done, warm, wall, res, per_step


# --------------------------------------------------------------------------------------------------
# exact-Shapley aggregation (config #5)
# --------------------------------------------------------------------------------------------------
def make_synthetic_table_device(n, begin, end, device):
    """Section 8(d) synthetic table restricted to masks [begin, end), generated on device (not timed)."""
    import numpy as np
    import torch
    s = torch.from_numpy(np.random.default_rng(0).uniform(100, 1000, size=n)).to(device)
    idx = torch.arange(begin, end, device=device, dtype=torch.int64)
    acc = torch.zeros(end - begin, dtype=torch.float64, device=device)
    for i in range(n):
        acc += ((idx >> i) & 1).double() * s[i]
    V = 1.0 - torch.exp(-acc / (s.sum() / 4.0))
    g = torch.Generator(device=device)
    g.manual_seed(1)
    V += 1e-3 * (torch.rand(end - begin, dtype=torch.float64, device=device, generator=g) * 2 - 1)
    if begin == 0:
        V[0] = 0.0
    return V.contiguous()


def bench_shapley(n, steps, warmup, rank, world):
    import torch
    import torch.distributed as dist
    from mplc.shapley import ShapleyAggregator, shard_range
    begin, end = shard_range(n, rank, world)
    dev = torch.device("cuda", torch.cuda.current_device())
    V = make_synthetic_table_device(n, begin, end, dev)
    agg = ShapleyAggregator(n, device=dev, count=end - begin)
    stream = torch.cuda.current_stream()
    for _ in range(warmup):
        p = agg.partial(V, begin)
        if world > 1:
            dist.all_reduce(p)
        agg.finalize(p)
    barrier(world)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        agg.partial(V, begin)
        ev[i][1].record(stream)
        if world > 1:
            dist.all_reduce(agg.partial_buf)
        agg.finalize(agg.partial_buf)
    barrier(world)
    wall = max_over_ranks(time.perf_counter() - t0, world)
    kern_ms = max_over_ranks(sum(a.elapsed_time(b) for a, b in ev) / steps, world)
    ms_per_step = wall * 1000 / steps
    shard_bytes = (end - begin) * 8
    achieved = shard_bytes / (kern_ms / 1000) / 1e9
    del V
    return {
        "metric": "exact-Shapley aggregation GB/s at N=%d" % n, "value": round((1 << n) * 8 / (ms_per_step / 1000) / 1e9, 2),
        "unit": "GB/s", "ms_per_step": round(ms_per_step, 4), "n": n, "table_bytes": (1 << n) * 8,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "shapley_block_kernel+shapley_reduce_blocks_kernel", "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": shard_bytes},
    }


def cpu_baseline_shapley(n_sample=24):
    from oracle import shapley as osh
    threads = host_threads()
    V = osh.synthetic_table(n_sample)
    osh.shapley_bitmask_f64_omp(n_sample, V, threads)
    reps, t0 = 0, time.perf_counter()
    while True:
        osh.shapley_bitmask_f64_omp(n_sample, V, threads)
        reps += 1
        if time.perf_counter() - t0 > 3.0 or reps >= 50:
            break
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(V.nbytes / dt / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"oracle fp64 OpenMP single pass over a 2^{n_sample} fp64 table ({V.nbytes >> 20} MiB), {reps} reps"}


# --------------------------------------------------------------------------------------------------
# training leg (config #3)
# --------------------------------------------------------------------------------------------------
def build_scenario(partners, epochs, M, G, early_stopping=False, signal=0.0):
    from mplc.dataset import Mnist
    from mplc.scenario import Scenario
    amounts = [1.0 / partners] * partners
    if partners == 10:
        amounts = [0.1] * 10
    sc = Scenario(partners, amounts, dataset=Mnist(synthetic=True, signal=signal), minibatch_count=M,
                  gradient_updates_per_pass_count=G, epoch_count=epochs, is_early_stopping=early_stopping)
    return sc.provision()


def _time_unit(fn, min_s=1.0, max_reps=50):
    fn()  # first call pays allocator / thread-pool start
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        if time.perf_counter() - t0 >= min_s or reps >= max_reps:
            break
    return (time.perf_counter() - t0) / reps


def cpu_baseline_train(sc, epochs, M):
    """CPU baseline for config #3: the oracle (torch-CPU fp32 restatement of the
    reference's Keras path, sequential, one coalition at a time, a fresh Keras Adam per partner fit) on the
    host's CPU share.  A whole 1023-coalition sweep takes hours on CPU, and one coalition of every size
    class still takes many minutes, so the bounded sample (~30 s) times the UNITS a sequential sweep is made
    of and sums them over every coalition in closed form:
      t_fit    one partner's FedAvg round: fresh model + Adam, ~9 Keras steps at bs_p on its minibatch
               (mplc/multi_partner_learning.py:301-334), averaged over the partners
      t_agg(k) the data-volume np.average of k models (mplc/mpl_utils.py:90-102), linear in k
      t_val    one evaluate on the 6000-sample val set; t_test one evaluate on the 10000-sample test set
      t_epoch  one singleton epoch: full partner data at bs_p, persistent Adam (:238-269)
    lean:      |S|>=2: E*M*(|S|*t_fit + t_agg(|S|)) + t_test;   |S|=1: E*t_epoch + t_test
    faithful:  adds the reference's per-round global-val evaluate and every partner fit's Keras
               validation_data evaluate, E*M*(|S|+1)*t_val (singletons: E*t_val)
    and checks the model against one real coalition {0,1} trained end to end (E=1, lean)."""
    import numpy as np
    import torch
    from math import comb
    from oracle import cnn as ocnn
    threads = host_threads()
    torch.set_num_threads(threads)
    t_all = time.perf_counter()
    ds = sc.dataset
    data = ocnn.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    prow = [p.train_idx for p in sc.partners_list]
    bs = [int(p.batch_size) for p in sc.partners_list]
    n = len(prow)
    sizes = np.array([len(r) for r in prow], dtype=np.float64)
    glob = ocnn.unpack(ocnn.init_params(ocnn.init_key(0, (1 << n) - 1)))
    fits = [0]

    def fit_round():
        p = fits[0] % n
        fits[0] += 1
        key = ocnn.shuffle_key(0, (1 << n) - 1, p)
        params = {k: v.clone() for k, v in glob.items()}
        opt = ocnn.KerasAdam(params)
        for rows in ocnn.fedavg_round_rows(key, prow[p], bs[p], M, 0, fits[0] % M):
            g, _ = ocnn.gradients(params, data.x_train[rows], data.y_train[rows])
            opt.step(params, g)
        return params

    t_fit = _time_unit(fit_round, min_s=3.0)
    models = [fit_round() for _ in range(n)]
    t_agg2 = _time_unit(lambda: ocnn.average_models(glob, models[:2], sizes[:2] / sizes[:2].sum()), 0.5)
    t_aggn = _time_unit(lambda: ocnn.average_models(glob, models, sizes / sizes.sum()), 0.5)
    t_val = _time_unit(lambda: ocnn.evaluate(glob, data.x_val, data.y_val), 1.0, 5)
    t_test = _time_unit(lambda: ocnn.evaluate(glob, data.x_test, data.y_test), 1.0, 5)

    def single_epoch():
        params = {k: v.clone() for k, v in glob.items()}
        opt = ocnn.KerasAdam(params)
        for rows in ocnn.single_epoch_rows(ocnn.shuffle_key(0, 1, 0), prow[0], bs[0], 0):
            g, _ = ocnn.gradients(params, data.x_train[rows], data.y_train[rows])
            opt.step(params, g)
    t0 = time.perf_counter()
    single_epoch()
    t_epoch = time.perf_counter() - t0

    def t_agg(k):
        return t_agg2 + (t_aggn - t_agg2) * (k - 2) / max(1, n - 2)

    lean = faithful = 0.0
    for k in range(1, n + 1):
        if k == 1:
            c_lean = epochs * t_epoch + t_test
            c_faith = c_lean + epochs * t_val
        else:
            c_lean = epochs * M * (k * t_fit + t_agg(k)) + t_test
            c_faith = c_lean + epochs * M * (k + 1) * t_val
        lean += comb(n, k) * c_lean
        faithful += comb(n, k) * c_faith
    # model check: one real coalition, E=1, lean schedule, end to end
    t0 = time.perf_counter()
    ocnn.coalition_value(data, prow, bs, (0, 1), epochs=1, M=M)
    t_pair = time.perf_counter() - t0
    pair_model = M * (2 * t_fit + t_agg(2)) + t_test
    n_coal = 2 ** n - 1
    return {"value": round(n_coal / lean, 5), "unit": "coalition evals/s", "cores": threads, "kind": "port",
            "faithful_value": round(n_coal / faithful, 6),
            "method": "unit-timed closed-form sum over all coalitions (bench.py cpu_baseline_train docstring)",
            "sample": (f"oracle torch-CPU fp32, {threads} threads, {time.perf_counter() - t_all:.0f}s of CPU work: "
                       f"t_fit {t_fit * 1e3:.0f} ms/partner-round, t_agg {t_agg2 * 1e3:.0f}-{t_aggn * 1e3:.0f} ms "
                       f"(2-{n} models), t_val {t_val:.2f}s, t_test {t_test:.2f}s, singleton epoch {t_epoch:.2f}s; "
                       f"sweep (E={epochs}, M={M}, {n_coal} coalitions) lean {lean:.0f}s, reference-faithful "
                       f"(+ per-round global-val and per-fit validation_data evals) {faithful:.0f}s; "
                       f"check: coalition (0,1) at E=1 measured {t_pair:.1f}s vs modelled {pair_model:.1f}s")}


def bench_train(args, rank, world):
    import numpy as np
    from mplc.contributivity import Contributivity
    from mplc.profiling import KernelTimer
    sc = build_scenario(args.partners, args.epochs, args.minibatches, args.gupp, args.early_stopping,
                        args.mnist_signal)
    from mplc.engine import CoalitionEngine
    sc.engine = CoalitionEngine.for_scenario(sc)
    eng = sc.engine
    if args.compact_share is not None:  # early-stopping batch compaction threshold (0: off; mplc/cnn.py)
        eng.compact_live_share = args.compact_share
    eng.warmup()  # untimed: code-object load (no training launch, so rocprof averages = timed launches)

    def progress(s, total, R):  # heartbeat for long sweeps (E=40: one sweep is several minutes)
        if s % 600 == 0 and total > 1000:
            log(f"train: lockstep step {s}/{total} ({R} replicas)")
    eng.progress = progress
    n = args.partners
    n_coal = 2 ** n - 1
    log(f"train leg ready: {n} partners, {n_coal} coalitions")

    def one_step():
        sc.coalition_values = {}  # retrain every coalition each step
        c = Contributivity(scenario=sc)
        c.compute_contributivity("Shapley values")
        return c

    timer = KernelTimer("all", TRAIN_KERNELS, stash=True, per_launch=("dense1_bwd_adam",))
    reps0 = [None]
    n_on = [0]

    def timed_step(i, planned):
        # the in-stream kernel timer (an event pair around every launch) runs on the first half of the timed
        # steps only; the second half runs without events, so the line shows what the timer itself costs
        if reps0[0] is None:
            reps0[0] = eng.stats["replicas"]
        on = not args.no_kernel_timer and (i < max(1, (planned + 1) // 2))
        eng.profiler = timer if on else None
        eng.time_test_eval = on  # the test evaluation's time, on the timer-on sweeps (one sync per batch)
        n_on[0] += int(on)
        return one_step()

    # reserve: the N=28 aggregation leg (~10 s with its table), at N=1 the bounded CPU baselines (~40 s + ~15 s)
    # and the config #4 sub-leg (one CIFAR10 TMCS run: ~110 s on one GPU)
    # (measured on the box, round 3: aggregation 1.3 s, CPU baselines 13 s + 6 s, the CIFAR run 107 s)
    # and the config #2 sub-leg (Titanic: a warm-up and a few sub-second sweeps, its CPU baseline 10 s)
    # and the reference-tutorial sub-leg (engine set-up, a warm-up and three 1.7 s sweeps)
    reserve = ((0 if args.no_shapley_agg else 10) + (25 if (world == 1 and not args.no_cpu_baseline) else 0) + 15
               + (0 if args.no_cifar else CIFAR_SUBLEG_S / world + 15 + (15 if world == 1 else 0))
               + (0 if args.no_titanic else 15 + (12 if world == 1 and not args.no_cpu_baseline else 0))
               + (0 if args.no_tutorial else 25))
    steps, warm, wall, c, per_step = run_budgeted(one_step, timed_step, args, world, reserve, "train")
    eng.profiler = None
    units = eng.model_impl.algorithmic_units(timer.stash)
    kernels = kernel_table(timer, units)
    split = dense1_split(eng, timer)
    if split:
        kernels["dense1_bwd_adam"]["split"] = split
    timer.stash = []
    local_reps = eng.stats["replicas"] - reps0[0]
    samples = units.get("samples", 0.0) / max(1, n_on[0]) * steps  # the stash covers the timer-on steps
    ms_per_step = wall * 1000 / steps
    total_train_samples = sum_over_ranks(samples, world)
    # the roofline kernel: the one with the largest share of the step's kernel time
    if args.no_kernel_timer:  # counter-collection passes (scripts/gpu_profile.sh): no events in the stream
        kernels = {}
        samples = steps * args.epochs * sum(eng.partner_sizes) * (2 ** (n - 1)) / world
        total_train_samples = sum_over_ranks(samples, world)
    on_ms, off_ms = per_step[:n_on[0]], per_step[n_on[0]:]
    timer_note = {"steps_with_kernel_timer": n_on[0],
                  "test_eval_ms_per_step": round(1000 * eng.stats.get("test_eval_s", 0.0) / max(1, n_on[0]), 1),
                  "ms_per_step_timer_on": round(1000 * sum(on_ms) / len(on_ms), 1) if on_ms else None,
                  "ms_per_step_timer_off": round(1000 * sum(off_ms) / len(off_ms), 1) if off_ms else None,
                  "note": "value covers every timed step; the kernels table and roofline come from the timer-on steps"}
    dom = max((k for k in kernels if "frac" in kernels[k]), key=lambda k: kernels[k]["ms_total"], default=None)
    kd = kernels.get(dom, {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None,
                           "launches": 0, "ms_avg": None, "time_share": None, "units_per_launch": None})
    roof = {"bound": kd["bound"], "achieved": kd["achieved"], "peak": kd["peak"], "unit": kd["unit"],
            "frac": kd["frac"], "traffic": None, "kernel": f"{dom}_kernel", "launches": kd["launches"],
            "kernel_ms_avg": kd["ms_avg"], "time_share": kd["time_share"]}
    if dom is None:
        roof["note"] = "in-stream kernel timing off (--no-kernel-timer)"
    elif kd["bound"] == "hbm":
        roof["algorithmic_bytes_per_launch"] = kd["units_per_launch"]
        roof["note"] = ("the step's dominant kernel; achieved = its algorithmic HBM bytes (" + KERNEL_UNITS[dom][3] +
                        ", counted per launch from the step's own schedule) / in-stream kernel time (HIP events "
                        "on the launch stream)")
    else:
        roof["algorithmic_flop_per_launch"] = kd["units_per_launch"]
        roof["note"] = ("the step's dominant kernel; achieved = " + KERNEL_UNITS[dom][3] + " / in-stream kernel time")
    out = {
        "metric": "coalition v(S) evals/sec (MNIST FedAvg)",
        "value": round(n_coal * steps / wall, 3), "unit": "coalition evals/s", "n_gpus": world,
        "steps": steps, "warmup": warm, "ms_per_step": round(ms_per_step, 1), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (MNIST-shaped: x~U[0,1) fp32 [60000,28,28,1], random one-hot labels)",
        "config": {"workload": f"BASELINE config #3: MNIST CNN, {n} partners random split, FedAvg, exact Shapley "
                               f"over all {n_coal} coalitions (E={args.epochs} fixed, M={args.minibatches}, "
                               f"G={args.gupp}), coalitions LPT-sharded x{world}",
                   "partners": n, "coalitions": n_coal, "epochs": args.epochs, "minibatch_count": args.minibatches,
                   "gradient_updates_per_pass": args.gupp, "batch_size": [int(p.batch_size) for p in sc.partners_list],
                   "replicas_trained_per_step": int(sum_over_ranks(local_reps, world) / max(1, steps)),
                   "train_samples_per_step": int(total_train_samples / steps),
                   "parallelism": f"coalition-shard x{world}"},
        "budget": {"budget_s": args.budget_s, "steps_requested": args.steps, "warmup_requested": args.warmup,
                   "timed_wall_s": round(wall, 2), "note": "one step = one whole 1023-coalition sweep; K clamped to "
                                                          "the whole steps that fit the wall-clock budget"},
        "roofline": roof,
        "kernels": kernels,
        "kernel_timer": timer_note,
        "shapley_values": [round(float(v), 6) for v in c.contributivity_scores],
        # coalition evaluations as the reference counts them, and the realised epochs (fixed E,
        # early stopping off, so every coalition trains exactly E epochs)
        "first_charac_fct_calls_count": int(c.first_charac_fct_calls_count),
        "epochs_per_coalition": args.epochs,
    }
    if args.early_stopping:
        # the reference's defaults (E=40, early stopping, mplc/constants.py:10-12): realised epochs per coalition,
        # the per-epoch val evaluations the stopping rule needs, and the lockstep batch's idle replica-steps
        # (stopped coalitions wait for the batch's last one)
        ep = np.array(eng.last_epochs_done, dtype=np.float64)
        st_ = eng.stats
        out["early_stopping"] = {
            "epochs_max": args.epochs, "realised_epochs_mean": round(float(ep.mean()), 2),
            "realised_epochs_min": int(ep.min()), "realised_epochs_max": int(ep.max()),
            "realised_epochs_hist": {str(int(k)): int(v) for k, v in zip(*np.unique(ep, return_counts=True))},
            "val_eval_s_per_step": round(st_.get("es_val_s", 0.0) / max(1, steps + warm), 2),
            "val_eval_share": round(st_.get("es_val_s", 0.0) / max(1e-9, (steps + warm) * ms_per_step / 1000), 4),
            "replica_steps_idle_share": round(1 - st_.get("replica_steps_live", 0) / max(1, st_.get("replica_steps", 1)),
                                              4),
            "replica_steps": int(st_.get("replica_steps", 0)), "replica_steps_live": int(st_.get("replica_steps_live", 0)),
            "compactions": int(st_.get("compactions", 0)),
            "compact_live_share": float(getattr(eng, "compact_live_share", eng.trainer.COMPACT_LIVE_SHARE)),
            "data": f"learnable synthetic MNIST (class templates, signal {args.mnist_signal})"}
        out["epochs_per_coalition"] = None
        out["config"]["workload"] = out["config"]["workload"].replace(f"E={args.epochs} fixed",
                                                                      f"E<={args.epochs} + early stopping")
    # whole-job algorithmic rate: training 2*E*sum n_p samples x 71.57 MFLOP + test evaluation
    # 1023 x 10000 x 23.98 MFLOP (MNIST CNN forward / train FLOPs per sample)
    job_flop = total_train_samples / steps * MNIST_TRAIN_FLOP + n_coal * len(sc.dataset.x_test) * MNIST_FWD_FLOP
    out["algorithmic"] = {"flop_per_step": int(job_flop), "tflops": round(job_flop / (ms_per_step / 1000) / 1e12, 2),
                          "frac_of_fp32_mfma_peak": round(job_flop / (ms_per_step / 1000) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)}
    return out, sc


# --------------------------------------------------------------------------------------------------
# CIFAR10 TMCS/SMCS leg (config #4)
# --------------------------------------------------------------------------------------------------
def build_cifar_scenario(epochs, signal, partners=20):
    import numpy as np
    from mplc.dataset import Cifar10
    from mplc.scenario import Scenario
    # [0.05]*20 fails the reference's sum check: the last share is 1 - the others
    amounts = [1.0 / partners] * (partners - 1)
    amounts.append(float(1 - np.sum(amounts)))
    sc = Scenario(partners, amounts, dataset=Cifar10(synthetic=True, signal=signal), minibatch_count=20,
                  gradient_updates_per_pass_count=8, epoch_count=epochs, is_early_stopping=False)
    return sc.provision()


def cifar_kernel_table(timer, units):
    """Config #4's per-kernel table (as kernel_table for config #3): launches, in-stream ms, time share, and for
    the convolutions (their algorithm's FLOPs: Winograd for conv2..conv4; conv1, under the ridge, its HBM bytes with
    the FLOP rate beside) and the W5 kernels (HBM bytes, CifarModel.algorithmic_units) the achieved rate against the
    roofline."""
    from mplc.cifar import BYTES_PER_SAMPLE as CIFAR_BYTES_PER_SAMPLE
    from mplc.cifar import FLOP_PER_SAMPLE, KERNEL_IDS
    tot = sum(timer.total_ms(k) for k in KERNEL_IDS) or 1.0
    out = {}
    for k in KERNEL_IDS:
        ms, n = timer.total_ms(k), timer.launches(k)
        e = {"launches": n, "ms_total": round(ms, 1), "ms_avg": round(ms / max(1, n), 4), "time_share": round(ms / tot, 4)}
        if ms > 0 and units:
            if k in CIFAR_BYTES_PER_SAMPLE:  # under the ridge (conv1, K = 27): HBM-bound; the MFMA rate beside it
                amount = units["samples"] * CIFAR_BYTES_PER_SAMPLE[k]
                rate, peak, unit, bound = amount / (ms / 1000) / 1e9, HBM_PEAK_GBS, "GB/s", "hbm"
                desc = (f"{k}'s compulsory HBM bytes ({CIFAR_BYTES_PER_SAMPLE[k]} per sample: "
                        f"{FLOP_PER_SAMPLE[k] / CIFAR_BYTES_PER_SAMPLE[k]:.1f} flop/B, under the "
                        f"{FP32_MFMA_PEAK_TFLOPS / HBM_PEAK_GBS * 1000:.1f} flop/B ridge)")
                mf = units["samples"] * FLOP_PER_SAMPLE[k] / (ms / 1000) / 1e12
                e["mfma_rate"] = {"achieved": round(mf, 2), "unit": "TFLOP/s", "frac": round(mf / FP32_MFMA_PEAK_TFLOPS, 4)}
            elif k in FLOP_PER_SAMPLE:
                amount = units["samples"] * FLOP_PER_SAMPLE[k]
                rate, peak, unit, bound = amount / (ms / 1000) / 1e12, FP32_MFMA_PEAK_TFLOPS, "TFLOP/s", "mfma"
                desc = f"{k}'s fp32 multiply-adds ({FLOP_PER_SAMPLE[k]} per sample)"
            elif f"{k}_bytes" in units:
                amount = units[f"{k}_bytes"]
                rate, peak, unit, bound = amount / (ms / 1000) / 1e9, HBM_PEAK_GBS, "GB/s", "hbm"
                desc = f"{k}'s algorithmic HBM bytes (W5 + RMSprop state by optimizer step, per-sample rows)"
            else:
                out[k] = e
                continue
            e.update({"bound": bound, "achieved": round(rate, 2), "peak": peak, "unit": unit,
                      "frac": round(rate / peak, 4), "units_per_launch": int(amount / max(1, n)), "algorithmic": desc})
        out[k] = e
    return out


def cpu_baseline_cifar(sc, coalitions, epochs, M):
    """Oracle (torch-CPU fp32, sequential like the reference) on a bounded sample: one singleton and one
    pair; FedAvg cost is linear in |S|, so the evaluated coalition list is extrapolated from t(1), t(2)."""
    import torch
    from oracle import cifar_cnn as occ
    threads = host_threads()
    torch.set_num_threads(threads)
    ds = sc.dataset
    data = occ.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    prow = [p.train_idx for p in sc.partners_list]
    bs = [p.batch_size for p in sc.partners_list]
    times = {}
    for k in (1, 2):
        t0 = time.perf_counter()
        occ.coalition_value(data, prow, bs, tuple(range(k)), epochs=epochs, M=M)
        times[k] = time.perf_counter() - t0
    per_partner = times[2] / 2.0
    total = sum(times[1] if len(c) == 1 else per_partner * len(c) for c in coalitions)
    return {"value": round(len(coalitions) / total, 5), "unit": "coalition evals/s", "cores": threads, "kind": "port",
            "sample": (f"oracle torch-CPU fp32 sequential fits (E={epochs}, M={M}) of |S|=1: {times[1]:.1f}s and |S|=2: "
                       f"{times[2]:.1f}s; the {len(coalitions)} coalitions this TMCS run evaluated extrapolated "
                       f"linearly in |S|: {total:.0f}s")}


CIFAR_TIMER_EVERY = 1  # config #4: the in-stream timer on every lockstep batch of the profile pass (bench_cifar)
CIFAR_SUBLEG_S = 115.0  # one config #4 TMCS run on one MI355X (round-2 measurement: 107 s)


def bench_cifar(args, rank, world, sub=False):
    """Config #4 (CIFAR10 TMCS/SMCS).  sub=True: the sub-leg of the default bench line - exactly one timed
    TMCS run, no warm-up step (the code object is loaded by eng.warmup(); each lockstep batch allocates its
    own buffers anyway)."""
    import numpy as np
    from mplc.cifar import DIRECT_FLOP_PER_SAMPLE, FLOP_PER_SAMPLE
    from mplc.contributivity import Contributivity
    from mplc.engine import CoalitionEngine
    from mplc.profiling import KernelTimer, StashOnly
    sc = build_cifar_scenario(args.cifar_epochs, args.signal, args.cifar_partners)
    if args.mc_plan_overhead is not None:  # planner experiments: the speculation budget (mplc.mc.plan_frontier)
        sc.mc_plan_overhead = args.mc_plan_overhead
    sc.engine = CoalitionEngine.for_scenario(sc)
    eng = sc.engine
    eng.warmup()

    from mplc.cifar import KERNEL_IDS as CIFAR_KERNEL_IDS
    timer = KernelTimer("all", list(CIFAR_KERNEL_IDS), stash=True)
    s0 = [0]
    sampled = {"batches": 0, "timed": 0, "timed_replica_steps": 0, "replica_steps": 0}

    prof = {"on": False}

    def progress(s, total, R):
        """Batch start: heartbeat on stderr, and in the profile pass the in-stream timer's batch sampling.  An
        event record around every launch costs about 15 % of this leg's wall time (its kernels are 40-340 us and a
        timing event flushes between them), and a timed batch runs as ONE lockstep batch on one stream - so the
        timer runs in a profile pass of the same (deterministic) TMCS job before the timed step, and the timed
        step runs every batch as the product does (two HIP streams, no events).  The kernels table and roofline
        come from the profile pass (its own launches and stashed schedules); `value` from the timed step."""
        if s != 0:
            return
        log(f"cifar: batch of {R} replicas, {total} steps, {eng.stats['coalitions']} coalitions so far")
        if not prof["on"]:
            return
        on = sampled["batches"] % CIFAR_TIMER_EVERY == 0
        eng.profiler = timer if on else None
        sampled["batches"] += 1
        sampled["replica_steps"] += R * total
        if on:
            sampled["timed"] += 1
            sampled["timed_replica_steps"] += R * total
    eng.progress = progress

    def one_step():
        sc.coalition_values = {}
        np.random.seed(0)
        c = Contributivity(scenario=sc)
        c.compute_contributivity(args.method)
        return c

    # under rocprofv3 --pmc (no HIP events): every step's schedule stashed, so that the counters' bytes of ALL
    # launches can be set beside the algorithmic bytes of the same launches (scripts/pmc_traffic.py)
    stash_all = StashOnly(args.cifar_profile_kernel) if args.no_kernel_timer else None

    def profile_step():  # the warm-up: the same job with the in-stream timer on (progress())
        prof["on"] = not args.no_kernel_timer
        try:
            return one_step()
        finally:
            prof["on"] = False
            eng.profiler = None

    def timed_step(i, planned):
        if s0[0] == 0:
            eng.profiler = stash_all  # None (no events in the timed steps) unless counters are being collected
            eng.time_test_eval = True
            s0[0] = eng.stats["samples"] or -1
        return one_step()

    # the profile pass is the warm-up step; without the timer (counter passes) there is none
    n_warm = 0 if args.no_kernel_timer else 1
    if sub:
        steps, warm, wall, c, _ = run_budgeted(profile_step, timed_step, args, world, 0, "cifar", max_steps=1,
                                               warmup=n_warm)
    else:
        reserve = (60 if (world == 1 and not args.no_cpu_baseline) else 0) + 15
        steps, warm, wall, c, _ = run_budgeted(profile_step, timed_step, args, world, reserve, "cifar",
                                               warmup=max(n_warm, min(args.warmup, 1)))
    eng.profiler = None
    units = eng.model_impl.algorithmic_units(timer.stash)
    timer.stash = []
    kernels = cifar_kernel_table(timer, units) if not args.no_kernel_timer else {}
    algorithmic_all = None
    if stash_all is not None and stash_all.stash:
        from mplc.cifar import compulsory_bytes
        ua = eng.model_impl.algorithmic_units(stash_all.stash)
        n_all = len(stash_all.stash)  # one launch of every training kernel per step
        algorithmic_all = {"launches": n_all, "samples_per_launch": ua["samples"] / n_all,
                           **{k.replace("_bytes", "_kernel"): v / n_all for k, v in ua.items() if k.endswith("_bytes")},
                           # every kernel's compulsory bytes (mplc.cifar.compulsory_bytes), totals over the run's
                           # training steps and evaluations, beside the counters' totals in scripts/pmc_traffic.py
                           "compulsory": compulsory_bytes(stash_all.stash, stash_all.evals),
                           "evaluations": len(stash_all.evals)}
        stash_all.stash, stash_all.evals = [], []
    kern_ms = timer.total_ms(args.cifar_profile_kernel)
    launches = timer.launches(args.cifar_profile_kernel)
    samples = eng.stats["samples"] - max(0, s0[0])
    # the timed batches' own samples (the stash), not the run's: the timer samples lockstep batches
    flops = (units["samples"] if units else 0) * FLOP_PER_SAMPLE[args.cifar_profile_kernel]
    achieved = flops / (kern_ms / 1000) / 1e12 if kern_ms > 0 else 0.0
    evals = c.first_charac_fct_calls_count
    coals = [k for k in c.charac_fct_values if len(k)]
    if getattr(args, "dump_values", None) and rank == 0:
        # every coalition value this run trained (counted and speculative) as bitmask -> v(S): input of the
        # planner simulations (scripts/sim_tmcs_planning.py)
        cache = dict(sc.coalition_values)
        cache.update({k: v for k, v in c.charac_fct_values.items() if len(k)})
        masks = np.array([sum(1 << i for i in k) for k in cache], dtype=np.int64)
        np.savez(args.dump_values, masks=masks, values=np.array(list(cache.values()), dtype=np.float64),
                 counted=np.array([sum(1 << i for i in k) for k in coals], dtype=np.int64))
    out = {
        "metric": f"coalition v(S) evals/sec (CIFAR10 FedAvg, {args.method})",
        "value": round(evals * steps / wall, 3), "unit": "coalition evals/s", "n_gpus": world,
        "steps": steps, "warmup": warm, "ms_per_step": round(wall * 1000 / steps, 1),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (CIFAR10-shaped: x = 0.4 class template + 0.6 U[0,1) fp32 [50000,32,32,3], one-hot labels)",
        "config": {"workload": f"BASELINE config #4: CIFAR10 CNN, {args.cifar_partners} partners, FedAvg, {args.method} (reference defaults, "
                               f"numpy seed 0), E={args.cifar_epochs} fixed, M=20, G=8, coalitions LPT-sharded x{world}",
                   "partners": args.cifar_partners, "method": args.method, "coalitions_evaluated": evals,
                   "coalition_sizes": {str(k): sum(1 for c_ in coals if len(c_) == k)
                                       for k in range(1, args.cifar_partners + 1)},
                   "train_samples_per_step_this_rank": int(samples / max(1, steps)),
                   "shapley_estimate": [round(float(v), 5) for v in c.contributivity_scores],
                   # planning (mplc.mc.plan_frontier / adaptive waves): coalitions trained vs counted by the
                   # estimator; the difference is speculation the sequential loop did not ask for
                   "coalitions_trained": int(eng.stats.get("coalitions", 0) // max(1, steps + warm)),
                   "frontier_plan": getattr(c, "plan_stats", None),
                   "sampling_iterations": getattr(c, "sampling_iterations", None),  # SMCS / WR_SMC to the stop rule
                   "replicas_per_launch": eng.stats.get("replicas", 0) / max(1, eng.stats.get("batches", 1)),
                   "lockstep_batches": eng.stats.get("batches", 0),
                   "test_eval_s": round(eng.stats.get("test_eval_s", 0.0), 2),
                   "parallelism": f"coalition-shard x{world}"},
        "budget": {"budget_s": args.budget_s, "steps_requested": args.steps, "warmup_requested": args.warmup,
                   "timed_wall_s": round(wall, 2)},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                     "kernel": args.cifar_profile_kernel, "launches": launches,
                     "kernel_ms_avg": round(kern_ms / max(1, launches), 4),
                     "algorithmic_flop_per_launch": int(flops / max(1, launches)),
                     "flop_per_sample": FLOP_PER_SAMPLE[args.cifar_profile_kernel],
                     "direct_equivalent_tflops": round(achieved * DIRECT_FLOP_PER_SAMPLE[args.cifar_profile_kernel]
                                                       / FLOP_PER_SAMPLE[args.cifar_profile_kernel], 2),
                     "note": "achieved = the kernel's own (Winograd F(2x2,3x3)) fp32 multiply-adds / in-stream "
                             "kernel time; direct_equivalent_tflops prices the same time at the direct "
                             "convolution's count"},
        "kernels": kernels,
        "algorithmic_bytes_per_launch_all": algorithmic_all,
        "kernel_timer": {"batches_timed": sampled["timed"], "batches": sampled["batches"],
                         "replica_steps_timed": sampled["timed_replica_steps"],
                         "replica_steps": sampled["replica_steps"],
                         "streams": eng.concurrent_batches,
                         "note": "in-stream HIP events around every launch of every lockstep batch of the profile "
                                 "pass (the warm-up step: the same deterministic TMCS job), each batch then run as ONE "
                                 "batch on one stream; the timed step runs without events, every batch in two halves "
                                 "on two HIP streams (the CIFAR10 default: CnnBatchTrainer.run_concurrent)"},
    }
    # the roofline on the step's dominant kernel (largest share of the kernel time), as the config #3 line
    dom = max((k for k in kernels if "frac" in kernels[k]), key=lambda k: kernels[k]["ms_total"], default=None)
    if dom is not None:
        kd = kernels[dom]
        wl = out["config"]["workload"]
        for k, e in kernels.items():  # PMC bytes per launch (all launches of the profiled run) beside the table
            pe = pmc_entry(f"{k}_kernel", wl) if e.get("bound") == "hbm" else None
            if pe is not None:
                e["traffic_pmc"] = int(pe["traffic_bytes_per_launch"])
                if pe.get("algorithmic_bytes_per_launch"):
                    e["traffic_over_algorithmic"] = round(pe["traffic_bytes_per_launch"] / pe["algorithmic_bytes_per_launch"], 4)
            pb = pmc_by_launch(k, wl)  # every kernel, either bound: counter bytes / compulsory bytes, all launches
            if pb is not None and pb.get("traffic_over_compulsory"):
                e["pmc_traffic_over_compulsory"] = round(pb["traffic_over_compulsory"], 4)
        out["roofline_conv2_fwd"] = out["roofline"]
        out["roofline"] = {"bound": kd["bound"], "achieved": kd["achieved"], "peak": kd["peak"], "unit": kd["unit"],
                           "frac": kd["frac"], "traffic": kd.get("traffic_pmc"),
                           "traffic_over_algorithmic": kd.get("traffic_over_algorithmic"),
                           "traffic_source": "profiles/pmc_traffic_config4.json: FETCH_SIZE x2 + WRITE_SIZE per launch "
                                             "over all launches of a --pmc run of this leg, beside the algorithmic bytes "
                                             "of the same launches" if kd.get("traffic_pmc") else None,
                           "kernel": dom, "launches": kd["launches"],
                           "kernel_ms_avg": kd["ms_avg"], "time_share": kd["time_share"],
                           "units_per_launch": kd["units_per_launch"],
                           "note": "the step's dominant kernel; achieved = " + kd["algorithmic"] +
                                   " / in-stream kernel time (HIP events on the launch stream)"}
    return out, sc, coals


# --------------------------------------------------------------------------------------------------
# Titanic leg (config #2)
# --------------------------------------------------------------------------------------------------
REFERENCE_TITANIC_EVALS_S = 10.1  # BASELINE.md / SURVEY 6: the reference's FedAvg + sklearn LR, measured in the build
                                  # container (60 random coalitions |S| >= 2, one CPU thread); not a published number


def build_titanic_scenario(partners=10, epochs=3, M=1):
    from mplc.dataset import Titanic
    from mplc.scenario import Scenario
    return Scenario(partners, [1.0 / partners] * partners if partners != 10 else [0.1] * 10,
                    dataset=Titanic(synthetic=True), epoch_count=epochs, minibatch_count=M,
                    is_early_stopping=False).provision()


def cpu_baseline_titanic(sc, coalitions, epochs, max_s=10.0):
    """The oracle (oracle/lr.py: every partner fit solved exactly by float64 Newton, the reference's sequential
    FedAvg: each of the E rounds refits every partner, np.average with data-volume weights, test accuracy) on one
    host thread, coalitions in a fixed shuffled order until max_s seconds: evals/s of that sample."""
    import numpy as np
    from oracle import lr as olr
    parts = [(np.asarray(p.x_train, dtype=np.float64), np.asarray(p.y_train)) for p in sc.partners_list]
    xte, yte = np.asarray(sc.dataset.x_test, dtype=np.float64), np.asarray(sc.dataset.y_test)
    order = np.random.default_rng(0).permutation(len(coalitions))
    done, t0 = 0, time.perf_counter()
    for i in order:
        coal = coalitions[i]
        sizes = [len(parts[p][1]) for p in coal]
        for _ in range(epochs):  # the M=1 rounds: every partner refits (warm start, same optimum) then the average
            thetas = [olr.fit_exact(*parts[p]) for p in coal]
            theta = np.average(np.array(thetas), axis=0, weights=np.asarray(sizes) / np.sum(sizes))
        olr.accuracy(theta, xte, yte)
        done += 1
        if time.perf_counter() - t0 > max_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 3), "unit": "coalition evals/s", "cores": 1, "kind": "port",
            "sample": f"{done} of the {len(coalitions)} coalitions (fixed shuffled order), oracle/lr.py exact fits, "
                      f"E={epochs} rounds each, {dt:.1f}s",
            "reference_measured": {"value": REFERENCE_TITANIC_EVALS_S, "unit": "coalition evals/s", "cores": 1,
                                   "note": "the reference's own FedAvg orchestration with sklearn lbfgs LR on this "
                                           "shape, 60 random coalitions |S| >= 2, timed in the build container "
                                           "(BASELINE.md, SURVEY 6)"}}


def bench_titanic(args, rank, world, sub=False):
    """Config #2: Titanic-shaped data, 10 partners, FedAvg logistic regression (E=3, M=1 as the reference's e2e
    test), exact "Shapley values" over all 1023 coalitions; one step = one full compute_contributivity (a fresh
    coalition cache each time).  Every coalition's whole FedAvg runs in one workgroup of one launch
    (csrc/logreg.hip), so the step is launch- and latency-bound, not a roofline kernel."""
    import torch
    from mplc.contributivity import Contributivity
    from mplc.engine import CoalitionEngine
    sc = build_titanic_scenario(10, 3, 1)
    sc.engine = CoalitionEngine.for_scenario(sc)

    def one_step():
        sc.coalition_values = {}
        c = Contributivity(scenario=sc)
        c.compute_contributivity("Shapley values")
        torch.cuda.synchronize()
        return c

    steps_max = 10 if sub else None
    steps, warm, wall, c, per_step = run_budgeted(one_step, lambda i, n: one_step(), args, world, 0, "titanic",
                                                  max_steps=steps_max, warmup=1)
    coals = [k for k in c.charac_fct_values if len(k)]
    out = {"metric": "coalition v(S) evals/sec (Titanic FedAvg LR, exact Shapley)",
           "value": round(c.first_charac_fct_calls_count * steps / wall, 2), "unit": "coalition evals/s",
           "n_gpus": world, "steps": steps, "warmup": warm, "ms_per_step": round(wall * 1000 / steps, 2),
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (Titanic-shaped: sklearn make_classification(887, 27, n_informative=8, random_state=0))",
           "config": {"workload": "BASELINE config #2: Titanic-shaped, 10 partners x 0.1, FedAvg logistic regression "
                                  f"(E=3, M=1), exact Shapley over all 1023 coalitions, coalitions LPT-sharded x{world}",
                      "coalitions_evaluated": c.first_charac_fct_calls_count,
                      "shapley": [round(float(v), 6) for v in c.contributivity_scores],
                      "per_step_ms": [round(t * 1000, 2) for t in per_step]}}
    return out, sc, coals


# The reference's own published timing of this path: notebooks/tutorials/
# Tutorial-2_Add_contributivity_measurement.ipynb, exact "Shapley values" on MNIST, 3 partners [0.001, 0.699, 0.3],
# E=10, M=3 (7 coalitions): "Computation time" 1525.8 s on a Colab GPU (model not printed), real MNIST
REFERENCE_TUTORIAL_S, REFERENCE_TUTORIAL_COALITIONS = 1525.8, 7
# and Tutorial-1_Run_your_first_scenario.ipynb: one FedAvg fit of the grand coalition, MNIST at 10 % (partners
# 874 / 2186 / 1312 rows), [0.2, 0.5, 0.3], E=10, M=3: "Training and evaluation on multiple partners: done.
# (179.283 seconds)" (per-epoch validation and the final test evaluation included)
REFERENCE_TUTORIAL1_FIT_S = 179.283


def bench_tutorial(args, rank, world, sub=False):
    """The reference tutorial's exact-Shapley experiment (the only published timing of this path):
    MNIST-shaped synthetic data at the full MNIST sizes (54,000 train / 6,000 val / 10,000 test rows), 3 partners
    [0.001, 0.699, 0.3], E=10, M=3, G=8 (the reference defaults; early stopping cannot act within 10 epochs at patience
    10), "Shapley values" over the 7 coalitions.  vs_baseline = this line's evals/s over the tutorial's 7 / 1525.8 s."""
    import torch
    from mplc.contributivity import Contributivity
    from mplc.dataset import Mnist
    from mplc.engine import CoalitionEngine
    from mplc.scenario import Scenario
    sc = Scenario(3, [0.001, 0.699, 0.3], dataset=Mnist(synthetic=True, signal=0.2), epoch_count=10,
                  minibatch_count=3).provision()
    sc.engine = CoalitionEngine.for_scenario(sc)

    def one_step():
        sc.coalition_values = {}
        c = Contributivity(scenario=sc)
        c.compute_contributivity("Shapley values")
        torch.cuda.synchronize()
        return c

    steps, warm, wall, c, per_step = run_budgeted(one_step, lambda i, n: one_step(), args, world, 0, "tutorial",
                                                  max_steps=3 if sub else None, warmup=1)
    value = c.first_charac_fct_calls_count * steps / wall
    ref = REFERENCE_TUTORIAL_COALITIONS / REFERENCE_TUTORIAL_S
    # Tutorial-1's timed fit: the grand coalition's FedAvg learning with its history (per-epoch validation, final
    # test evaluation), as Scenario.run() starts; a warm-up, then the median of three
    sc1 = Scenario(3, [0.2, 0.5, 0.3], dataset=Mnist(synthetic=True, signal=0.2), epoch_count=10, minibatch_count=3,
                   dataset_proportion=0.1).provision()
    sc1.engine = CoalitionEngine.for_scenario(sc1)

    def fit_once():
        mpl = sc1.multi_partner_learning_approach(sc1, is_save_data=False, record_history=True)
        mpl.fit()
        torch.cuda.synchronize()
        return mpl

    fit_once()
    fit_s = []
    for _ in range(3):
        t0 = time.perf_counter()
        mpl1 = fit_once()
        fit_s.append(time.perf_counter() - t0)
    fit_med = sorted(fit_s)[1]
    sc1.engine.release()
    out = {"metric": "coalition v(S) evals/sec (reference Tutorial-2: MNIST exact Shapley, 3 partners, E=10, M=3)",
           "value": round(value, 4), "unit": "coalition evals/s", "n_gpus": world, "steps": steps, "warmup": warm,
           "ms_per_step": round(wall * 1000 / steps, 1), "higher_is_better": True, "scaling": "strong",
           "vs_baseline": round(value / ref, 1), "dtype": "f32",
           "data": "synthetic (MNIST-shaped, learnable: class templates at signal 0.2, the full MNIST sizes; the "
                   "tutorial ran real MNIST)",
           "config": {"workload": "reference Tutorial-2 (notebooks/tutorials/Tutorial-2_Add_contributivity_measurement"
                                  ".ipynb): MNIST CNN, 3 partners [0.001, 0.699, 0.3], FedAvg, E=10, M=3, G=8, exact "
                                  f"Shapley over the 7 coalitions, coalitions LPT-sharded x{world}",
                      "batch_size": [p.batch_size for p in sc.partners_list],
                      "coalitions_evaluated": c.first_charac_fct_calls_count,
                      "shapley": [round(float(v), 6) for v in c.contributivity_scores],
                      "per_step_ms": [round(t * 1000, 1) for t in per_step],
                      "baseline": {"value": round(ref, 5), "unit": "coalition evals/s",
                                   "source": "the tutorial notebook's printed computation time, 1525.8 s for 7 "
                                             "coalitions on a Colab GPU (BASELINE.md section 1)"},
                      "tutorial1_fit": {"seconds": round(fit_med, 4), "runs_s": [round(t, 4) for t in fit_s],
                                        "reference_s": REFERENCE_TUTORIAL1_FIT_S,
                                        "speedup": round(REFERENCE_TUTORIAL1_FIT_S / fit_med, 1),
                                        "batch_size": [p.batch_size for p in sc1.partners_list],
                                        "test_accuracy": round(float(mpl1.history.score), 4),
                                        "workload": "Tutorial-1_Run_your_first_scenario.ipynb: one FedAvg fit of "
                                                    "the grand coalition, MNIST-shaped at 10 % (874 / 2186 / 1312 "
                                                    "rows), E=10, M=3, with per-epoch validation and the final test "
                                                    "evaluation"}}}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--budget-s", type=float, default=480.0,
                    help="wall-clock budget from process start for the whole run (driver limit: 600 s)")
    ap.add_argument("--leg", default="train", choices=["train", "shapley", "cifar", "titanic", "tutorial", "dist-check"])
    ap.add_argument("--method", default="TMCS")
    ap.add_argument("--signal", type=float, default=0.4)
    ap.add_argument("--cifar-epochs", type=int, default=1)
    ap.add_argument("--cifar-partners", type=int, default=20)
    ap.add_argument("--cifar-profile-kernel", default="conv2_fwd")
    ap.add_argument("--partners", type=int, default=10)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--minibatches", type=int, default=20)
    ap.add_argument("--gupp", type=int, default=8)
    ap.add_argument("--n", type=int, default=28)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-shapley-agg", action="store_true")
    ap.add_argument("--no-cifar", action="store_true", help="leave out the config #4 sub-leg of the default line")
    ap.add_argument("--no-titanic", action="store_true", help="leave out the config #2 sub-leg of the default line")
    ap.add_argument("--no-tutorial", action="store_true",
                    help="leave out the reference-tutorial sub-leg (vs its published timing) of the default line")
    ap.add_argument("--early-stopping", action="store_true",
                    help="train leg at the reference's stopping rule (with --epochs 40: its defaults)")
    ap.add_argument("--mnist-signal", type=float, default=0.0,
                    help="class-template signal of the synthetic MNIST (0: random labels)")
    ap.add_argument("--compact-share", type=float, default=None,
                    help="train leg: early-stopping batch compaction threshold (default mplc/cnn.py; 0 = off)")
    ap.add_argument("--dump-values", default=None, help="cifar leg: save the trained v(S) values (npz) here")
    ap.add_argument("--mc-plan-overhead", type=float, default=None,
                    help="cifar leg: TMCS speculation budget in replica-trainings per batch (default: the library's 8)")
    ap.add_argument("--no-kernel-timer", action="store_true",
                    help="no HIP events in the stream (rocprofv3 --pmc passes: counters only)")
    args = ap.parse_args()
    if os.environ.get("ROCPROF_COUNTER_COLLECTION", "").lower() in ("1", "true", "yes") and \
            not os.environ.get("MPLC_FORCE_KERNEL_TIMER"):
        # under `rocprofv3 --pmc` the in-stream HIP events are left out: round 2 saw rocprofv3's counter thread
        # crash (SIGSEGV) on a --pmc pass of this bench with an event record around every launch
        # (profiles/r03_pmc_events_crash.txt); the counter passes need the kernels, not the timer
        args.no_kernel_timer = True
        log("rocprofv3 counter collection detected: in-stream kernel timer off")
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # one child process per GPU; this process stays off the GPU
    rank, world, _ = dist_init(expected=args.gpus, use_gpu=args.leg != "dist-check")
    if args.leg == "dist-check":
        # the multi-rank plumbing alone (no GPU): every rank reports (rank, local rank) through one all_gather
        import torch
        import torch.distributed as dist
        mine = torch.tensor([rank, int(os.environ.get("LOCAL_RANK", "0"))], dtype=torch.int64)
        got = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        if world > 1:
            dist.all_gather(got, mine)
        else:
            got = [mine]
        if rank == 0:
            print(json.dumps({"leg": "dist-check", "n_gpus": world, "ranks": [g.tolist() for g in got],
                              "master": [os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")]}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    if args.leg == "shapley":
        out = bench_shapley(args.n, max(args.steps, 5), max(args.warmup, 2), rank, world)
        out.update({"n_gpus": world, "steps": max(args.steps, 5), "warmup": max(args.warmup, 2),
                    "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
                    "data": "synthetic", "config": {"workload": f"Synthetic v(S) table N={args.n} (2^{args.n} fp64), "
                                                                f"range-sharded + RCCL all-reduce x{world}"}})
        if rank == 0:
            out["cpu_baseline"] = cpu_baseline_shapley() if (world == 1 and not args.no_cpu_baseline) else None
    elif args.leg == "tutorial":
        out = bench_tutorial(args, rank, world)
        out["cpu_baseline"] = None
    elif args.leg == "titanic":
        out, sc, coals = bench_titanic(args, rank, world)
        if rank == 0:
            out["cpu_baseline"] = cpu_baseline_titanic(sc, coals, 3) if (world == 1 and not args.no_cpu_baseline) else None
    elif args.leg == "cifar":
        out, sc, coals = bench_cifar(args, rank, world)
        if rank == 0:
            out["cpu_baseline"] = (cpu_baseline_cifar(sc, coals, args.cifar_epochs, 20)
                                   if (world == 1 and not args.no_cpu_baseline) else None)
    else:
        out, sc = bench_train(args, rank, world)
        wl = out["config"]["workload"]
        out["roofline"]["traffic"] = pmc_traffic(out["roofline"]["kernel"], wl)
        for k, e in out["kernels"].items():  # PMC bytes per launch beside each kernel's algorithmic count
            if e.get("bound") == "hbm":
                e["traffic_pmc"] = pmc_traffic(f"{k}_kernel", wl)
        out["roofline"]["traffic_source"] = TRAFFIC_SOURCE
        if not args.no_shapley_agg:
            # the lockstep training batch's buffers are no longer needed: give the 2 GiB table room
            sc.engine.release()
            agg = bench_shapley(args.n, 10, 2, rank, world)
            agg["roofline"]["traffic"] = pmc_traffic("shapley_block_kernel", wl)
            agg["roofline"]["traffic_source"] = TRAFFIC_SOURCE
            # N = 20..26 are measured with `--leg shapley --n N` (scripts/gpu_bench.sh), not here:
            # the kernel-trace average of shapley_block_kernel must stay the N=28 launch
            out["shapley_agg"] = agg
            log(f"shapley_agg N={args.n}: {agg['value']} GB/s")
        if not args.no_cifar:
            # BASELINE config #4 in the same line: one CIFAR10 TMCS run (20 partners), its own roofline and CPU
            # baseline; the MNIST lockstep buffers are returned first
            sc.engine.release()
            c4, c4_sc, c4_coals = bench_cifar(args, rank, world, sub=True)
            if rank == 0:
                c4["cpu_baseline"] = (cpu_baseline_cifar(c4_sc, c4_coals, args.cifar_epochs, 20)
                                      if (world == 1 and not args.no_cpu_baseline) else None)
            for k in ("n_gpus", "higher_is_better", "scaling", "vs_baseline", "dtype", "budget", "warmup"):
                c4.pop(k, None)
            out["config4"] = c4
            log(f"config #4 sub-leg: {c4['value']} evals/s")
        if not args.no_titanic:
            # BASELINE config #2 in the same line: the Titanic LR exact-Shapley sweep (a few seconds)
            c2, c2_sc, c2_coals = bench_titanic(args, rank, world, sub=True)
            if rank == 0:
                c2["cpu_baseline"] = (cpu_baseline_titanic(c2_sc, c2_coals, 3)
                                      if (world == 1 and not args.no_cpu_baseline) else None)
            for k in ("n_gpus", "higher_is_better", "scaling", "vs_baseline", "budget"):
                c2.pop(k, None)
            out["config2"] = c2
            log(f"config #2 sub-leg: {c2['value']} evals/s")
        if not args.no_tutorial:
            # the reference's only published timing of this path (its Tutorial-2 exact-Shapley run), with
            # vs_baseline against it: a few seconds
            tut = bench_tutorial(args, rank, world, sub=True)
            for k in ("n_gpus", "higher_is_better", "scaling", "budget"):
                tut.pop(k, None)
            out["tutorial"] = tut
            log(f"tutorial sub-leg: {tut['value']} evals/s, {tut['vs_baseline']}x the reference's published run")
        if rank == 0:
            out["cpu_baseline"] = (cpu_baseline_train(sc, args.epochs, args.minibatches)
                                   if (world == 1 and not args.no_cpu_baseline) else None)
    out["wall_s_total"] = round(time.perf_counter() - T_PROC0, 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
