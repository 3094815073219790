"""Probe: per-replica-step cost vs lockstep batch size (HBM budget), config #3 shape, E=1.
python scripts/probe_scale.py n_coalitions size(0 = any size >= 2) budget_gb [budget_gb ...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))

import numpy as np
import torch

from mplc.dataset import Mnist
from mplc.engine import CoalitionEngine
from mplc.scenario import Scenario
from mplc.profiling import KernelTimer


def main():
    n = int(sys.argv[1])
    size = int(sys.argv[2])
    budgets = [float(b) for b in sys.argv[3:]] or [400]
    sc = Scenario(10, [0.1] * 10, dataset=Mnist(synthetic=True), minibatch_count=20, epoch_count=1,
                  is_early_stopping=False).provision()
    from itertools import combinations
    pool = [c for r in range(2, 11) for c in combinations(range(10), r)] if size == 0 else \
        list(combinations(range(10), size))
    rng = np.random.default_rng(0)
    pick = rng.choice(len(pool), size=min(n, len(pool)), replace=False)
    coals = sorted(pool[i] for i in pick)
    n = len(coals)
    for b in budgets:
        eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=int(b * (1 << 30)))
        t_start = [time.time()]

        def progress(s, total, R):
            torch.cuda.synchronize()
            print(f"    step {s}/{total} R={R} t={time.time() - t_start[0]:.2f}s", flush=True)
        eng.progress = progress
        eng.evaluate(coals[:2])
        for kern in ("conv_bwd_data", "dense1_bwd_adam"):
            eng.profiler = KernelTimer(kern)
            torch.cuda.synchronize()
            t0 = time.time()
            t_start[0] = t0
            eng.evaluate(coals)
            torch.cuda.synchronize()
            dt = time.time() - t0
            ms = eng.profiler.total_ms()
            nb = len(eng.plan_batches(coals))
            reps = sum(len(c) for c in coals)
            print(f"budget {b:6.1f} GB: {nb} batches, {reps} replicas: {dt:6.2f}s total, {kern} {ms:8.1f} ms "
                  f"({ms * 1000 / (reps * 180):.2f} us per replica-step)", flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
