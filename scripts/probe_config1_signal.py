"""CPU probe (oracle only): v(S) of config #1's partitions (the reference's contrib yml: proportion 0.1, E=1,
M=10, G=8; and the 3-partner [0.2, 0.5, 0.3] variant) on synthetic MNIST at several class-template signals, to
pick a signal where the models have learned but are not saturated (tests/test_config1_gpu.py)."""
import sys
import time

import numpy as np

sys.path.insert(0, "distributed-learning-contributivity_amd")
sys.path.insert(0, ".")
from mplc.dataset import Mnist  # noqa: E402
from mplc.scenario import Scenario  # noqa: E402
from oracle import cnn as ocnn  # noqa: E402

for signal in [float(s) for s in sys.argv[1:]] or [0.1, 0.2]:
    for amounts in ([0.1, 0.9], [0.2, 0.5, 0.3]):
        sc = Scenario(len(amounts), amounts, dataset=Mnist(synthetic=True, signal=signal), dataset_proportion=0.1,
                      minibatch_count=10, gradient_updates_per_pass_count=8, epoch_count=1)
        sc.provision()
        ds = sc.dataset
        data = ocnn.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
        prow = [p.train_idx for p in sc.partners_list]
        bs = [p.batch_size for p in sc.partners_list]
        n = len(amounts)
        out = []
        for r in range(1, n + 1):
            from itertools import combinations
            for k in combinations(range(n), r):
                t0 = time.time()
                out.append((k, round(float(ocnn.coalition_value(data, prow, bs, k, seed=0, epochs=1, M=10)[0]), 4),
                            round(time.time() - t0, 1)))
        print(signal, amounts, [len(r) for r in prow], bs, out, flush=True)
