"""Benchmark driver (contract: one JSON line on rank 0).

python bench.py [--gpus N] [--steps K] [--warmup W] [--leg shapley|train]

leg "shapley": exact-Shapley aggregation of a synthetic N=28 v(S) table (2^28 fp64 = 2 GiB, resident
in HBM before timing), range-sharded across ranks, partial sums all-reduced over RCCL.  One step = one
full aggregation.  metric = algorithmic GB/s (8 bytes per mask read once).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "distributed-learning-contributivity_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def dist_init():
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return rank, world, local


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


def cpu_baseline_shapley(n_sample=24):
    """Oracle fp64 OpenMP single pass over a 2^24 table (bounded sample, ~128 MiB), GB/s."""
    from oracle import shapley as osh
    threads = min(16, os.cpu_count() or 1)
    V = osh.synthetic_table(n_sample)
    osh.shapley_bitmask_f64_omp(n_sample, V, threads)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        osh.shapley_bitmask_f64_omp(n_sample, V, threads)
        reps += 1
        if time.perf_counter() - t0 > 3.0 or reps >= 50:
            break
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(V.nbytes / dt / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"oracle fp64 OpenMP single pass over a 2^{n_sample} fp64 table ({V.nbytes >> 20} MiB), "
                      f"{reps} reps"}


def bench_shapley(args, rank, world):
    import torch
    import torch.distributed as dist
    from mplc.shapley import ShapleyAggregator, shard_range
    n = args.n
    begin, end = shard_range(n, rank, world)
    dev = torch.device("cuda", torch.cuda.current_device())
    V = make_synthetic_table_device(n, begin, end, dev)
    agg = ShapleyAggregator(n, device=dev, count=end - begin)
    stream = torch.cuda.current_stream()

    def step():
        p = agg.partial(V, begin)
        if world > 1:
            dist.all_reduce(p)
        return agg.finalize(p)

    for _ in range(args.warmup):
        step()
    barrier(world)
    # kernel-only timing with HIP events on the launch stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        agg.partial(V, begin)
        ev[i][1].record(stream)
        if world > 1:
            dist.all_reduce(agg.partial_buf)
        agg.finalize(agg.partial_buf)
    barrier(world)
    wall = time.perf_counter() - t0
    wall = max_over_ranks(wall, world)
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    kern_ms = max_over_ranks(kern_ms, world)
    ms_per_step = wall * 1000 / args.steps
    total_bytes = (1 << n) * 8
    value = total_bytes / (ms_per_step / 1000) / 1e9
    shard_bytes = (end - begin) * 8
    achieved = shard_bytes / (kern_ms / 1000) / 1e9
    out = {
        "metric": "exact-Shapley aggregation GB/s at N=%d" % n,
        "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "Synthetic v(S) table, N=%d partners (2^%d fp64), range-sharded + RCCL all-reduce" % (n, n),
                   "n": n, "table_bytes": total_bytes, "parallelism": "range-shard x%d" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "shapley_block_kernel+reduce", "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": shard_bytes},
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--leg", default="shapley", choices=["shapley"])
    ap.add_argument("--n", type=int, default=28)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    rank, world, _ = dist_init()
    out = bench_shapley(args, rank, world)
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_shapley()
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
