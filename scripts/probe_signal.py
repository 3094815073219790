"""Probe: v(S) of CIFAR10-shaped template data vs signal level and coalition size (config #4 shape, E=1).
python scripts/probe_signal.py sig1 [sig2 ...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "distributed-learning-contributivity_amd"))
import numpy as np

from mplc.dataset import Cifar10
from mplc.engine import CoalitionEngine
from mplc.scenario import Scenario

for sig in [float(a) for a in sys.argv[1:]]:
    ds = Cifar10(synthetic=True, signal=sig)
    sc = Scenario(20, [0.05] * 19 + [float(1 - np.sum([0.05] * 19))], dataset=ds, minibatch_count=20,
                  epoch_count=1, is_early_stopping=False).provision()
    eng = CoalitionEngine.for_scenario(sc)
    coals = [(0,), (1,), (0, 1), (2, 3), tuple(range(4)), tuple(range(8)), tuple(range(12)), tuple(range(20))]
    t0 = time.time()
    v = eng.evaluate(coals)
    print(f"signal {sig}: " + ", ".join(f"|S|={len(c)}:{x:.3f}" for c, x in zip(coals, v)) + f"  ({time.time() - t0:.1f}s)",
          flush=True)
