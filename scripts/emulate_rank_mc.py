"""Emulate an N-GPU config #4 TMCS run on a single GPU (record and replay, every rank).

An N-rank run plans TMCS waves N times longer (Contributivity._truncated_loop: mc_wave_scale = world size) and
LPT-shards every frontier batch over the ranks (mplc.parallel.sharded_evaluate); the estimator itself runs
SPMD on every rank.  On one GPU:
  1. run the whole job with mc_wave_scale = N, recording every batch the estimator requested and the time
     spent training it (the rest of the wall time is host work every rank repeats: walks, planning, the
     stopping rule);
  2. replay: train every rank's LPT share of each recorded batch (v(S) is a deterministic function of
     (S, seed), so the shares are exactly the coalitions each rank would train), timed.
job time ~ host time of 1. + the sum over batches of the slowest rank's training time in 2.  (The all_reduce of each batch's values - a few KB over
xGMI - is not included.)
python scripts/emulate_rank_mc.py N [method] [mc_plan_overhead|-] [mc_wave_scale]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))
import threading

import numpy as np
import torch

import bench

_T0 = time.time()


def _heartbeat():  # a line on stderr every 30 s: a long shard is not a hung GPU command
    while True:
        time.sleep(30)
        print(f"heartbeat {time.time() - _T0:.0f}s", file=sys.stderr, flush=True)


threading.Thread(target=_heartbeat, daemon=True).start()
from mplc import parallel

N = int(sys.argv[1])
METHOD = sys.argv[2] if len(sys.argv) > 2 else "TMCS"
OVERHEAD = float(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3] != "-" else None  # mc_plan_overhead
WAVE = int(sys.argv[4]) if len(sys.argv) > 4 else N  # mc_wave_scale (the product uses the world size)
batches, train_s = [], [0.0]


def recording(evaluate_local, coalitions, partner_sizes, device=None, **_):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vals = np.asarray(evaluate_local(coalitions), dtype=np.float64)
    torch.cuda.synchronize()
    train_s[0] += time.perf_counter() - t0
    batches.append(list(coalitions))
    return vals


parallel.sharded_evaluate = recording
torch.cuda.set_device(0)
sc = bench.build_cifar_scenario(1, 0.4)
sc.mc_wave_scale = WAVE
if OVERHEAD is not None:
    sc.mc_plan_overhead = OVERHEAD
from mplc.contributivity import Contributivity
from mplc.engine import CoalitionEngine
sc.engine = CoalitionEngine.for_scenario(sc)
sc.engine.warmup()
eng = sc.engine
eng.evaluate([(0,), (0, 1)])  # one-time device allocation outside the timing
sc.coalition_values = {}
np.random.seed(0)
torch.cuda.synchronize()
t0 = time.perf_counter()
c = Contributivity(scenario=sc)
c.compute_contributivity(METHOD)
torch.cuda.synchronize()
wall = time.perf_counter() - t0
host = wall - train_s[0]
evals = c.first_charac_fct_calls_count
trained = sum(len(b) for b in batches)
print(f"[{METHOD} N={N} overhead={OVERHEAD} wave_scale={WAVE}] full job on 1 GPU: {wall:.1f} s ({train_s[0]:.1f} s training, {host:.1f} s host), "
      f"{len(batches)} batches, {trained} coalitions trained, {evals} evaluated by the estimator", flush=True)
sizes = eng.partner_sizes
# replay: every rank's LPT share of every batch, timed; the N-rank job waits at each batch's all_reduce for its
# slowest rank, so its training time is the sum over batches of the max over ranks
per_rank = np.zeros(N)
synced, reps = 0.0, np.zeros(N)
for b in batches:
    shards = parallel.lpt_shard([parallel.coalition_cost(k, sizes) for k in b], N)
    times = np.zeros(N)
    for r, shard in enumerate(shards):
        if not shard:
            continue
        mine = [b[i] for i in shard]
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        eng.evaluate(mine)
        torch.cuda.synchronize()
        times[r] = time.perf_counter() - t1
        reps[r] += sum(len(k) for k in mine)
    per_rank += times
    synced += times.max()
job = host + synced
print(f"[{METHOD} N={N}] emulated job: {job:.1f} s = host {host:.1f} s + sum over batches of the slowest rank's "
      f"training {synced:.1f} s (ranks' own totals {np.round(per_rank, 1).tolist()}, replicas per rank "
      f"{reps.astype(int).tolist()}, {reps.mean() / max(1, len(batches)):.0f} per batch) -> whole-job value "
      f"{evals / job:.2f} evals/s", flush=True)
