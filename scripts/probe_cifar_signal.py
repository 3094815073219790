"""CPU probe (oracle only): CIFAR10 v(S) on config #4's partition shape (20 partners of 1822 rows, bs 11, M=20,
G=8) at several class-template signals and epoch counts, to pick a regime where the coalitions have LEARNED
(accuracy >= 0.5) but are not saturated (tests/test_cifar_gpu.py::test_config4_learned_accuracies_vs_oracle)."""
import sys
import time

import numpy as np

sys.path.insert(0, "distributed-learning-contributivity_amd")
sys.path.insert(0, ".")
from mplc.dataset import Cifar10  # noqa: E402
from mplc.scenario import Scenario  # noqa: E402
from oracle import cifar_cnn as occ  # noqa: E402

coals = [tuple(int(c) for c in s.split(",")) for s in (__import__("os").environ.get("COALS") or "3;0,7;2,9,14").split(";")]
for arg in sys.argv[1:]:
    signal, epochs = (float(arg.split(":")[0]), int(arg.split(":")[1]))
    amounts = [0.05] * 19 + [float(1 - np.sum([0.05] * 19))]
    sc = Scenario(20, amounts, dataset=Cifar10(synthetic=True, signal=signal), minibatch_count=20,
                  gradient_updates_per_pass_count=8, epoch_count=epochs, is_early_stopping=False).provision()
    ds = sc.dataset
    data = occ.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    prow = [p.train_idx for p in sc.partners_list]
    bs = [p.batch_size for p in sc.partners_list]
    out = []
    for k in coals:
        t0 = time.time()
        out.append((k, round(float(occ.coalition_value(data, prow, bs, k, seed=0, epochs=epochs, M=20)[0]), 4),
                    round(time.time() - t0, 1)))
    print(signal, epochs, out, flush=True)
