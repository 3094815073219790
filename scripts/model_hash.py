"""Bit-identity probe: train a config-shaped batch of coalitions and print the sha1 of every final model row and of
v(S).  python scripts/model_hash.py [mnist|cifar] [n_coalitions] [epochs]   (A/B of two library + host trees)"""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))

import numpy as np  # noqa: E402

from mplc.dataset import Cifar10, Mnist  # noqa: E402
from mplc.engine import CoalitionEngine  # noqa: E402
from mplc.scenario import Scenario  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "cifar"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    E = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    if which == "cifar":
        P, amounts, ds = 20, [0.05] * 19 + [float(1 - np.sum([0.05] * 19))], Cifar10(synthetic=True, signal=0.4)
    else:
        P, amounts, ds = 10, [0.1] * 10, Mnist(synthetic=True, signal=0.2)
    sc = Scenario(P, amounts, dataset=ds, minibatch_count=20, gradient_updates_per_pass_count=8, epoch_count=E,
                  is_early_stopping=False).provision()
    eng = CoalitionEngine.for_scenario(sc)
    rng = np.random.default_rng(1)
    coals = sorted({tuple(sorted(rng.choice(P, size=int(rng.integers(1, 6)), replace=False).tolist()))
                    for _ in range(n)})
    res = eng.evaluate(coals, return_details=True, return_models=True)
    h = hashlib.sha1()
    for m in res["models"]:
        for w in m:
            h.update(np.ascontiguousarray(w, dtype=np.float32).tobytes())
    v = np.asarray(res["scores"], dtype=np.float64)
    print(f"{which}: {len(coals)} coalitions E={E} mean acc {v.mean():.4f} "
          f"models sha1 {h.hexdigest()[:16]} v sha1 {hashlib.sha1(v.tobytes()).hexdigest()[:12]}", flush=True)


if __name__ == "__main__":
    main()
