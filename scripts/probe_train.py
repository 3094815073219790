"""Probe: time the batched trainer on the BASELINE config #3 shape (10 partners, MNIST-shaped synthetic).
python scripts/probe_train.py [n_coalitions] [epochs] [size]"""
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    sc = Scenario(10, [0.1] * 10, dataset=Mnist(synthetic=True), minibatch_count=20, epoch_count=E,
                  is_early_stopping=False).provision()
    eng = CoalitionEngine.for_scenario(sc)
    from itertools import combinations
    pool = list(combinations(range(10), size))
    rng = np.random.default_rng(0)
    coals = sorted(pool[i] for i in rng.choice(len(pool), size=min(n, len(pool)), replace=False))
    n = len(coals)
    t0 = time.time()
    eng.evaluate(coals[:2])
    torch.cuda.synchronize()
    t1 = time.time()
    v = eng.evaluate(coals)
    torch.cuda.synchronize()
    t2 = time.time()
    reps = n * size
    print(f"warm {t1 - t0:.2f}s; {n} coalitions x {size} partners, E={E}: {t2 - t1:.2f}s "
          f"-> {n / (t2 - t1):.2f} evals/s, {reps / (t2 - t1):.1f} replica-epochs/s; mean acc {v.mean():.3f}",
          flush=True)


if __name__ == "__main__":
    main()
