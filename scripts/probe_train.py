"""Probe: time the batched trainer on a BASELINE shape.
python scripts/probe_train.py [n_coalitions] [epochs] [size] [mnist|cifar]
  mnist: config #3 shape (10 partners, MNIST-shaped synthetic, M=20)
  cifar: config #4 shape (20 partners, CIFAR10-shaped synthetic, M=20)"""
import hashlib
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))

import numpy as np
import torch

from mplc.dataset import Cifar10, Mnist
from mplc.engine import CoalitionEngine
from mplc.scenario import Scenario


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    which = sys.argv[4] if len(sys.argv) > 4 else "mnist"
    if which == "cifar":
        P, amounts, ds = 20, [0.05] * 19 + [float(1 - np.sum([0.05] * 19))], Cifar10(synthetic=True)
    else:
        P, amounts, ds = 10, [0.1] * 10, Mnist(synthetic=True)
    sc = Scenario(P, amounts, dataset=ds, minibatch_count=20, epoch_count=E, is_early_stopping=False).provision()
    eng = CoalitionEngine.for_scenario(sc)
    from itertools import combinations
    rng = np.random.default_rng(0)
    if size <= 5 or P <= 10:
        pool = list(combinations(range(P), size))
        coals = sorted(pool[i] for i in rng.choice(len(pool), size=min(n, len(pool)), replace=False))
    else:
        coals = sorted({tuple(sorted(rng.choice(P, size=size, replace=False).tolist())) for _ in range(n)})
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
          f"-> {n / (t2 - t1):.2f} evals/s, {reps / (t2 - t1):.1f} replica-epochs/s; mean acc {v.mean():.3f}; "
          f"bs {sorted(set(eng.batch_sizes))}, n_p {sorted(set(eng.partner_sizes))[:3]}; "
          f"v sha1 {hashlib.sha1(np.ascontiguousarray(v, dtype=np.float64).tobytes()).hexdigest()[:12]}", flush=True)


if __name__ == "__main__":
    main()
