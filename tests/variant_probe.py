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
    # cifar10_smallb: batches of at most 16 samples (M=6, G=8: 6 / 9 / 15), the size at which dense5_fwd runs its
    # 16-row form (the variant library runs the 32-row form there)
    for name, maker, amounts, M, G in (("mnist", digits_as_mnist, [0.2, 0.5, 0.3], 2, 4),
                                       ("cifar10", digits_as_cifar, [0.2, 0.5, 0.3], 2, 4),
                                       ("cifar10_smallb", digits_as_cifar, [0.2, 0.3, 0.5], 6, 8)):
        x, y = maker()
        ds = ArrayDataset(x[:1500], y[:1500], x[1500:], y[1500:], **({"name": "cifar10"} if "cifar" in name else {}))
        sc = Scenario(3, amounts, dataset=ds, minibatch_count=M, gradient_updates_per_pass_count=G,
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
