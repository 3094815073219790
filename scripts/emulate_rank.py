"""Emulate one rank of an N-GPU config #3 run on a single GPU: train only rank 0's LPT shard of the 1023
coalitions (no collective; the Shapley values are then meaningless) and time it, to check strong scaling
before the driver's multi-GPU run.  python scripts/emulate_rank.py N"""
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


def sharded_local(evaluate_local, coalitions, partner_sizes, device=None):
    shards = parallel.lpt_shard([parallel.coalition_cost(c, partner_sizes) for c in coalitions], N)
    vals = np.zeros(len(coalitions))
    mine = shards[0]
    if mine:
        vals[mine] = evaluate_local([coalitions[i] for i in mine])
    return vals


parallel.sharded_evaluate = sharded_local
torch.cuda.set_device(0)
sc = bench.build_scenario(10, 2, 20, 8)
from mplc.contributivity import Contributivity
from mplc.engine import CoalitionEngine
sc.engine = CoalitionEngine.for_scenario(sc)
sc.engine.warmup()
for _ in range(2):  # the first pass carries the one-time device allocation, as bench.py's warm-up step
    sc.coalition_values = {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    c = Contributivity(scenario=sc)
    c.compute_contributivity("Shapley values")
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
print(f"emulated rank 0 of {N}: {wall:.2f} s, replicas {sc.engine.stats['replicas']}, "
      f"-> whole-job value {1023 / wall:.2f} evals/s", flush=True)
