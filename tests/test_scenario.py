"""CPU: partner partitions, batch sizes and FedAvg weights are index-identical to the reference.

tests/golden/splits.json was produced by running the reference's Scenario.split_data /
compute_batch_sizes (mplc/scenario.py:571-724) and Dataset global splits (mplc/dataset.py:62-106) on
index-valued datasets of the BASELINE configs' sizes."""
import json
import os

import numpy as np
import pytest

from mplc.dataset import Dataset, Mnist
from mplc.scenario import Scenario
from mplc.fedavg import aggregation_weights
from mplc.cnn import minibatch_bounds, mix64 as host_mix64, init_key, shuffle_key
from oracle import cnn as ocnn

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "splits.json")


def load():
    with open(GOLDEN) as f:
        return json.load(f)["data"]


def make_dataset(rec):
    n, nt = rec["n_train_orig"], rec["n_test"]
    local = rec["dataset"] in ("mnist", "cifar10", "titanic")

    class IdxDataset(Dataset):
        if local:
            train_test_split_local = staticmethod(Mnist.train_test_split_local)
            train_val_split_local = staticmethod(Mnist.train_val_split_local)

    ncls = 2 if rec["dataset"] == "titanic" else 10
    x = np.arange(n, dtype=np.int64).reshape(-1, 1)
    y = np.eye(ncls, dtype="float32")[np.arange(n) % ncls]
    xt = np.arange(nt, dtype=np.int64).reshape(-1, 1)
    yt = np.eye(ncls, dtype="float32")[np.arange(nt) % ncls]
    return IdxDataset(rec["dataset"], (1,), ncls, x, y, xt, yt)


@pytest.mark.parametrize("rec", load(), ids=lambda r: r["tag"])
def test_split_matches_reference(rec):
    ds = make_dataset(rec)
    sc = Scenario(rec["partners_count"], rec["amounts"], dataset=ds, dataset_proportion=rec["dataset_proportion"],
                  minibatch_count=rec["minibatch_count"],
                  gradient_updates_per_pass_count=rec["gradient_updates_per_pass_count"], epoch_count=1)
    sc.provision()
    assert ds.x_train.ravel().tolist() == rec["x_train_global"]
    assert ds.x_val.ravel().tolist() == rec["x_val_global"]
    for p, gp in zip(sc.partners_list, rec["partners"]):
        assert p.x_train.ravel().tolist() == gp["x_train"]
        assert ds.x_train[p.train_idx].ravel().tolist() == gp["x_train"]
        assert p.batch_size == gp["batch_size"]


def test_amounts_that_fail_reference_assert():
    # [0.05]*20 fails np.sum(amounts) == 1 in the reference (mplc/scenario.py:587-590); so does the engine
    rec = [r for r in load() if r["tag"] == "cfg4_cifar_20p"][0]
    ds = make_dataset(rec)
    sc = Scenario(20, [0.05] * 20, dataset=ds, minibatch_count=20)
    with pytest.raises(AssertionError):
        sc.provision()


def test_minibatch_bounds_match_np_split():
    for n in (437, 3936, 4374, 4373, 57, 1822):
        for M in (1, 3, 10, 20):
            b = minibatch_bounds(n, M)
            split_indices = np.arange(1, M + 1) / M
            parts = np.split(np.arange(n), (split_indices[:-1] * n).astype(int))
            assert [len(p) for p in parts] == [b[i + 1] - b[i] for i in range(M)]


def test_aggregation_weights_match_reference_aggregators():
    sizes = [4374] * 9 + [4373]
    w, scl = aggregation_weights(sizes, "data-volume")
    ref = np.asarray(sizes) / np.sum(sizes)
    assert w == [float(v) for v in ref]
    assert scl == float(np.broadcast_to(ref, (1, 10)).swapaxes(-1, 0).sum(axis=0)[0])
    wu, _ = aggregation_weights([1, 2, 3], "uniform")
    assert wu == [1 / 3] * 3


def test_local_score_aggregation_is_rejected():
    """'local-score' is registered in the reference (mplc/mpl_utils.py:132-136) but its aggregator returns
    no weights (:118-128); the scenario refuses it up front."""
    import pytest
    from mplc.dataset import ArrayDataset, digits_as_mnist
    from mplc.scenario import Scenario
    x, y = digits_as_mnist()
    ds = ArrayDataset(x[:600], y[:600], x[600:800], y[600:800], name="mnist")
    with pytest.raises(NotImplementedError, match="local-score"):
        Scenario(2, [0.5, 0.5], dataset=ds, aggregation_weighting="local-score")


def test_host_and_oracle_keys_agree():
    for s in (0, 1, 12345):
        for mask in (1, 3, 1023, 0x3FF):
            assert init_key(s, mask) == ocnn.init_key(s, mask)
            for p in range(3):
                assert shuffle_key(s, mask, p) == ocnn.shuffle_key(s, mask, p)
    assert host_mix64(0) == ocnn.mix64(0)


def test_oracle_keyed_perm_is_a_permutation():
    for n in (1, 2, 3, 43, 44, 437, 4374, 30573):
        out = ocnn.keyed_perm(0x1234567 + n, n, np.arange(n))
        assert sorted(out.tolist()) == list(range(n))


def test_missing_dataset_is_an_error_not_synthetic(monkeypatch, tmp_path):
    """a missing mnist.npz / cifar10.npz / titanic.csv raises unless synthetic data are asked for
    (synthetic=True, or MPLC_SYNTHETIC_DATA=1 which logs a warning and flags results.csv)."""
    import pytest
    from mplc import dataset as dm
    monkeypatch.setenv("MPLC_DATA_DIR", str(tmp_path))
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.delenv("MPLC_SYNTHETIC_DATA", raising=False)
    for cls in (dm.Titanic,):
        with pytest.raises(FileNotFoundError):
            cls()
    with pytest.raises(FileNotFoundError):
        dm.Mnist(n_train=100, n_test=10)
    with pytest.raises(FileNotFoundError):
        dm.Cifar10(n_train=100, n_test=10)
    assert dm.Mnist(synthetic=True, n_train=100, n_test=10).synthetic
    monkeypatch.setenv("MPLC_SYNTHETIC_DATA", "1")
    assert dm.Titanic().synthetic


def test_label_codes_equal_reference_string_encoding():
    """split_data's label codes: LabelEncoder over str(row) per sample (reference mplc/scenario.py:573),
    computed once per distinct row."""
    import numpy as np
    from sklearn.preprocessing import LabelEncoder
    from mplc.scenario import _label_codes
    rng = np.random.default_rng(3)
    one_hot = np.eye(10, dtype=np.float32)[rng.integers(0, 10, 4000)]
    ints = rng.integers(0, 2, 900)
    for y in (one_hot, ints):
        ref = LabelEncoder().fit_transform([str(r) for r in y])
        assert np.array_equal(_label_codes(y), ref)
