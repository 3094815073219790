"""Run by tests/test_variants_gpu.py in a child process (MPLC_LIB_PATH selects the library build): trains small
MNIST and CIFAR10 FedAvg coalitions on the HIP engine and prints one JSON line with the sha1 of every final model
row and of the v(S) values.  Test infrastructure."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "distributed-learning-contributivity_amd")):
    sys.path.insert(0, p)


def main():
    import numpy as np
    from mplc import _native
    from mplc.dataset import ArrayDataset, digits_as_cifar, digits_as_mnist
    from mplc.engine import CoalitionEngine
    from mplc.scenario import Scenario
    out = {"lib": os.path.relpath(_native.lib_path(), REPO)}
    for name, maker in (("mnist", digits_as_mnist), ("cifar10", digits_as_cifar)):
        x, y = maker()
        ds = ArrayDataset(x[:1500], y[:1500], x[1500:], y[1500:], **({"name": "cifar10"} if name == "cifar10" else {}))
        sc = Scenario(3, [0.2, 0.5, 0.3], dataset=ds, minibatch_count=2, gradient_updates_per_pass_count=4,
                      epoch_count=2, is_early_stopping=False).provision()
        eng = CoalitionEngine.for_scenario(sc, memory_budget_bytes=4 << 30, eval_budget_bytes=1 << 30)
        res = eng.evaluate([(0,), (1, 2), (0, 1, 2)], return_details=True, return_models=True)
        h = hashlib.sha1()
        for m in res["models"]:
            for w in m:
                h.update(np.ascontiguousarray(w, dtype=np.float32).tobytes())
        out[name] = {"models_sha1": h.hexdigest()[:16], "scores": [float(v) for v in res["scores"]]}
    print("VARIANT_PROBE " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
