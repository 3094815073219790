"""Emulate rank 0 of an N-GPU config #4 TMCS run on a single GPU (record and replay).

An N-rank run plans TMCS waves N times longer (Contributivity._truncated_loop: mc_wave_scale = world size) and
LPT-shards every frontier batch over the ranks (mplc.parallel.sharded_evaluate); the estimator itself runs
SPMD on every rank.  On one GPU:
  1. run the whole job with mc_wave_scale = N, recording every batch the estimator requested and the time
     spent training it (the rest of the wall time is host work every rank repeats: walks, planning, the
     stopping rule);
  2. replay: train only rank 0's LPT share of each recorded batch (v(S) is a deterministic function of
     (S, seed), so the shares are exactly the coalitions rank 0 would train), timed.
rank 0's time ~ host time of 1. + training time of 2.  (The all_reduce of each batch's values - a few KB over
xGMI - is not included.)
python scripts/emulate_rank_mc.py N [method]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))
import numpy as np
import torch

import bench
from mplc import parallel

N = int(sys.argv[1])
METHOD = sys.argv[2] if len(sys.argv) > 2 else "TMCS"
batches, train_s = [], [0.0]


def recording(evaluate_local, coalitions, partner_sizes, device=None):
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
sc.mc_wave_scale = N
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
print(f"[{METHOD} N={N}] full job on 1 GPU: {wall:.1f} s ({train_s[0]:.1f} s training, {host:.1f} s host), "
      f"{len(batches)} batches, {trained} coalitions trained, {evals} evaluated by the estimator", flush=True)
sizes = eng.partner_sizes
rank0_train, rank0_reps = 0.0, 0
for b in batches:
    shard = parallel.lpt_shard([parallel.coalition_cost(k, sizes) for k in b], N)[0]
    if not shard:
        continue
    mine = [b[i] for i in shard]
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    eng.evaluate(mine, is_early_stopping=True)
    torch.cuda.synchronize()
    rank0_train += time.perf_counter() - t1
    rank0_reps += sum(len(k) for k in mine)
rank0 = host + rank0_train
print(f"[{METHOD} N={N}] emulated rank 0: {rank0:.1f} s ({rank0_train:.1f} s training {rank0_reps} replicas in "
      f"{len(batches)} batches = {rank0_reps / max(1, len(batches)):.0f} per batch, {host:.1f} s host) -> "
      f"whole-job value {evals / rank0:.2f} evals/s", flush=True)
