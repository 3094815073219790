"""Scenarios and oracle spreads shared by the accuracy gates of tests/test_config1_gpu.py and
tests/test_workload_gpu.py and by scripts/oracle_spread.py, which writes the fixtures
tests/golden/oracle_spread_<name>.json (the oracle's v(S) over many CPU thread counts, i.e. fp32 summation
orders, and in fp64).  Test infrastructure: it runs the oracle (oracle/cnn.py) only as the checker."""
import json
import os
import tempfile
import zlib
from itertools import combinations

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CONFIG3_COALS = [(p,) for p in range(10)] + [(2, 7), (0, 9), (4, 5), (1, 3), (6, 8), (0, 5), (2, 9), (3, 7)]


def config1_scenario(amounts, signal=0.3):
    """The scenario main.py builds from the contrib yml with `amounts` (synthetic MNIST as mnist.npz)."""
    from mplc.dataset import _synthetic_images
    from mplc.scenario import Scenario
    d = tempfile.mkdtemp(prefix="cfg1_")
    x, y, xt, yt = _synthetic_images((28, 28, 1), 60000, 10000, 0, signal)
    q = lambda a: np.round(a[..., 0] * 255).astype(np.uint8)  # noqa: E731  (the real file's uint8 pixels)
    np.savez(os.path.join(d, "mnist.npz"), x_train=q(x), y_train=np.argmax(y, 1).astype(np.uint8), x_test=q(xt),
             y_test=np.argmax(yt, 1).astype(np.uint8))
    old = os.environ.get("MPLC_DATA_DIR")
    os.environ["MPLC_DATA_DIR"] = d
    try:
        sc = Scenario(len(amounts), list(amounts), dataset_name="mnist", dataset_proportion=0.1,
                      samples_split_option=["basic", "random"], epoch_count=1, minibatch_count=10,
                      gradient_updates_per_pass_count=8).provision()
    finally:
        if old is None:
            os.environ.pop("MPLC_DATA_DIR", None)
        else:
            os.environ["MPLC_DATA_DIR"] = old
    return sc


def config3_scenario(epochs=1):
    from mplc.dataset import Mnist
    from mplc.scenario import Scenario
    return Scenario(10, [0.1] * 10, dataset=Mnist(synthetic=True, signal=0.2), minibatch_count=20,
                    gradient_updates_per_pass_count=8, epoch_count=epochs, is_early_stopping=False).provision()


# config #4's 20-partner CIFAR10 partition ([0.05] * 19 + [1 - 0.95]: the reference's sum check), signal 0.4, and the
# eight coalitions of tests/test_workload_gpu.py::test_config4_learned_accuracies_vs_oracle (fixed before any run)
CONFIG4_E2_COALS = [(2, 9, 14), (0, 7, 11, 16), (1, 4, 6, 11, 15, 19), (3, 5, 8, 10, 12), (2, 9, 14, 17),
                    (0, 3, 5, 8, 10, 12, 13, 18), (6, 13, 17), (1, 7, 15, 18)]


def config4_scenario(epochs=1):
    from mplc.dataset import Cifar10
    from mplc.scenario import Scenario
    amounts = [0.05] * 19 + [float(1 - np.sum([0.05] * 19))]
    return Scenario(20, amounts, dataset=Cifar10(synthetic=True, signal=0.4), minibatch_count=20,
                    gradient_updates_per_pass_count=8, epoch_count=epochs, is_early_stopping=False).provision()


# tests/test_ranking_gpu.py: the 10-partner exact-Shapley ranking scenario, chosen with scripts/probe_ranking.py
# (profiles/r06_probe_ranking_grid4.log: the ranking unchanged under five ~1-ulp perturbations of the training data,
# every adjacent Shapley gap >= 2.25x the spread of the difference): MNIST-shaped synthetic data (class templates,
# signal 0.25, 1000 test images), dataset_proportion 0.1, random split over unequal amounts (np.sum == 1.0 exactly,
# the reference's assert mplc/scenario.py:587-590), FedAvg E=4, M=1, G=32 (one round per epoch: the sequential CPU
# oracle's sweep of all 1023 coalitions is ~0.7 M optimizer steps)
RANKING = {"amounts": [0.02, 0.03, 0.04, 0.06, 0.08, 0.10, 0.12, 0.15, 0.18, 0.22], "signal": 0.25,
           "dataset_proportion": 0.1, "n_test": 1000, "epoch_count": 4, "minibatch_count": 1,
           "gradient_updates_per_pass_count": 32, "split": "random"}


def ranking_scenario():
    from mplc.dataset import Mnist
    from mplc.scenario import Scenario
    p = RANKING
    return Scenario(10, list(p["amounts"]), dataset=Mnist(synthetic=True, signal=p["signal"], n_test=p["n_test"]),
                    dataset_proportion=p["dataset_proportion"], samples_split_option=["basic", p["split"]],
                    minibatch_count=p["minibatch_count"],
                    gradient_updates_per_pass_count=p["gradient_updates_per_pass_count"],
                    epoch_count=p["epoch_count"], is_early_stopping=False).provision()


def scenario(name):
    if name == "config1_3p":
        sc = config1_scenario([0.2, 0.5, 0.3])
        return sc, [k for r in range(1, 4) for k in combinations(range(3), r)]
    if name == "config1_2p":
        return config1_scenario([0.1, 0.9]), [(0,), (1,), (0, 1)]
    if name == "config3":
        return config3_scenario(), CONFIG3_COALS
    if name == "config3_e2":  # the same partition and coalitions at E=2 (where the models have left the steep part)
        return config3_scenario(epochs=2), CONFIG3_COALS
    if name == "config4_e2":
        return config4_scenario(epochs=2), CONFIG4_E2_COALS
    raise ValueError(name)


def data_crc(sc):
    ds = sc.dataset
    c = zlib.crc32(np.ascontiguousarray(ds.x_train).tobytes())
    c = zlib.crc32(np.ascontiguousarray(np.asarray(ds.y_train)).tobytes(), c)
    c = zlib.crc32(np.ascontiguousarray(ds.x_test).tobytes(), c)
    for p in sc.partners_list:
        c = zlib.crc32(np.ascontiguousarray(p.train_idx, dtype=np.int64).tobytes(), c)
    return int(c)


def oracle_values(sc, coals, threads, precise=False, seed=0):
    """v(S) of `coals` from the scenario's model oracle (oracle/cnn.py for MNIST, oracle/cifar_cnn.py for CIFAR10,
    sequential like the reference) at `threads` CPU threads; precise=True: every tensor operation in fp64."""
    import torch
    from oracle import cnn as ocnn
    ds = sc.dataset
    cifar = getattr(ds, "name", "mnist") == "cifar10"
    if cifar:
        from oracle import cifar_cnn as occ
        data = occ.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    else:
        data = ocnn.Data(ds.x_train, ds.y_train, ds.x_val, ds.y_val, ds.x_test, ds.y_test)
    prow = [p.train_idx for p in sc.partners_list]
    bs = [p.batch_size for p in sc.partners_list]
    t0 = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        if cifar:
            if precise:
                raise NotImplementedError("oracle/cifar_cnn.py coalition_value has no fp64 mode")
            return [float(occ.coalition_value(data, prow, bs, k, seed=seed, epochs=sc.epoch_count,
                                              M=sc.minibatch_count)[0]) for k in coals]
        return [float(ocnn.coalition_value(data, prow, bs, k, seed=seed, epochs=sc.epoch_count, M=sc.minibatch_count,
                                           precise=precise)[0]) for k in coals]
    finally:
        torch.set_num_threads(t0)


def golden_split(tag):
    """The reference's own split of a BASELINE config (tests/golden/splits.json, made by make_golden.py)."""
    with open(os.path.join(GOLDEN, "splits.json")) as f:
        return next(r for r in json.load(f)["data"] if r["tag"] == tag)


def load_spread(name, sc=None):
    """The committed spread fixture of scenario `name` ({"coalitions", "fp32": {threads: values}, "fp64"});
    with `sc`, checked to belong to that scenario's data and partition."""
    with open(os.path.join(GOLDEN, f"oracle_spread_{name}.json")) as f:
        rec = json.load(f)
    if sc is not None:
        assert rec["data_crc32"] == data_crc(sc), f"oracle_spread_{name}.json was made for other data"
    return rec
