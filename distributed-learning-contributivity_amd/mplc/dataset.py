"""Datasets on the coalition path (mplc/dataset.py:37-106, 397-488).

Dataset keeps the reference's contract (name, input_shape, num_classes, x_/y_{train,val,test},
train_val_split_global 90/10 with random_state 42, shorten_dataset_proportion with np.random.seed(42),
local train/test and train/val splits for partners) so partner partitions are index-identical to the
reference's (tests/test_scenario.py against tests/golden/splits.json).

The images themselves: MNIST is loaded from a local keras-format ``mnist.npz`` (x_train, y_train,
x_test, y_test) found via $MPLC_DATA_DIR, ./data or ~/.keras/datasets - the reference downloads it
(mplc/dataset.py:415-440), which is impossible offline.  Without a local file, ``Mnist(synthetic=True)``
builds tensors of MNIST's exact shapes (x ~ U[0,1) float32 [60000,28,28,1], one-hot labels) for
throughput work; ``synthetic`` records which one was used.  Synthetic data are never substituted silently:
with ``synthetic=None`` (the default, and what Scenario(dataset_name=...) and the CLI use) a missing file
raises FileNotFoundError unless MPLC_SYNTHETIC_DATA=1 opts in, which logs a warning (and results.csv
carries a ``synthetic_data`` column).
"""
import logging
import os

import numpy as np
from sklearn.model_selection import train_test_split

from . import constants


class Dataset:
    def __init__(self, dataset_name, input_shape, num_classes, x_train, y_train, x_test, y_test):
        self.name = dataset_name
        self.input_shape = input_shape
        self.num_classes = num_classes
        self.x_train = x_train
        self.x_val = None
        self.x_test = x_test
        self.y_train = y_train
        self.y_val = None
        self.y_test = y_test
        # row ids of x_train in the ORIGINAL array, kept through the global splits (engine bookkeeping)
        self.train_rows = np.arange(len(x_train))
        self.train_val_split_global()

    def train_val_split_global(self):
        """mplc/dataset.py:62-69: 90/10 train/val, random_state=42."""
        if self.x_val is not None or self.y_val is not None:
            raise Exception("x_val and y_val should be of NoneType")
        ids = np.arange(len(self.x_train))
        tr, va = train_test_split(ids, test_size=0.1, random_state=42)
        self.x_train, self.x_val = self.x_train[tr], self.x_train[va]
        self.y_train, self.y_val = self.y_train[tr], self.y_train[va]

    @staticmethod
    def train_test_split_local(x, y):
        return x, np.array([]), y, np.array([])

    @staticmethod
    def train_val_split_local(x, y):
        return x, np.array([]), y, np.array([])

    def generate_new_model(self):
        raise NotImplementedError("models are built by the engine's batched kernels (mplc.engine)")

    def shorten_dataset_proportion(self, dataset_proportion):
        """mplc/dataset.py:83-106."""
        if dataset_proportion == 1:
            return
        if dataset_proportion < 0:
            raise ValueError("The dataset proportion should be strictly between 0 and 1")
        skip_train_idx = int(round(len(self.x_train) * dataset_proportion))
        train_idx = np.arange(len(self.x_train))
        skip_val_idx = int(round(len(self.x_val) * dataset_proportion))
        val_idx = np.arange(len(self.x_val))
        np.random.seed(42)
        np.random.shuffle(train_idx)
        np.random.shuffle(val_idx)
        self.x_train = self.x_train[train_idx[0:skip_train_idx]]
        self.y_train = self.y_train[train_idx[0:skip_train_idx]]
        self.x_val = self.x_val[val_idx[0:skip_val_idx]]
        self.y_val = self.y_val[val_idx[0:skip_val_idx]]


def _local_mnist():
    dirs = [os.environ.get("MPLC_DATA_DIR", ""), os.path.join(os.getcwd(), "data"),
            os.path.expanduser("~/.keras/datasets")]
    for d in dirs:
        p = os.path.join(d, "mnist.npz") if d else ""
        if p and os.path.exists(p):
            with np.load(p, allow_pickle=False) as f:
                return (f["x_train"], f["y_train"]), (f["x_test"], f["y_test"])
    return None


def _synthetic_allowed(synthetic, what):
    """True: build synthetic data.  synthetic=True asks for it; synthetic=None (no local file found) only
    with MPLC_SYNTHETIC_DATA=1; otherwise the missing file is an error, never a silent substitution."""
    if synthetic:
        return True
    if synthetic is None and os.environ.get("MPLC_SYNTHETIC_DATA", "") == "1":
        logging.getLogger("mplc").warning(f"{what} not found: using SYNTHETIC data of the same shape "
                                          "(MPLC_SYNTHETIC_DATA=1); the results do not describe the real dataset")
        return True
    raise FileNotFoundError(f"{what} not found (set MPLC_DATA_DIR, or pass synthetic=True / set "
                            "MPLC_SYNTHETIC_DATA=1 for shape-identical synthetic data); no network to download it")


def _one_hot(y, k):
    return np.eye(k, dtype="float32")[np.asarray(y, dtype=np.int64).ravel()]


def _synthetic_images(shape, n_train, n_test, seed, signal=0.0):
    """Dataset-shaped synthetic images, x in [0,1) float32, one-hot labels of 10 classes.  signal = 0: pure
    uniform noise with random labels (throughput work, every model at chance).  signal > 0: x = signal *
    template[y] + (1 - signal) * noise with one fixed random template per class, so accuracy grows with the
    amount of training data - truncated Monte-Carlo estimators then behave as on real data."""
    rng = np.random.default_rng(seed)
    y_train = rng.integers(0, 10, n_train)
    y_test = rng.integers(0, 10, n_test)
    x_train = rng.random((n_train,) + shape, dtype=np.float32)
    x_test = rng.random((n_test,) + shape, dtype=np.float32)
    if signal > 0:
        tmpl = np.random.default_rng(seed + 1).random((10,) + shape, dtype=np.float32)
        s = np.float32(signal)
        x_train = (s * tmpl[y_train] + (np.float32(1) - s) * x_train).astype(np.float32)
        x_test = (s * tmpl[y_test] + (np.float32(1) - s) * x_test).astype(np.float32)
    return x_train, _one_hot(y_train, 10), x_test, _one_hot(y_test, 10)


class Mnist(Dataset):
    """mplc/dataset.py:397-488 (model: the engine's batched CNN of the same architecture)."""

    def __init__(self, synthetic=None, seed=0, n_train=60000, n_test=10000, signal=0.0):
        self.img_rows = self.img_cols = 28
        loaded = None if synthetic else _local_mnist()
        if loaded is None:
            _synthetic_allowed(synthetic, "mnist.npz")
        if loaded is None and signal > 0:  # learnable: class templates + noise (see _synthetic_images)
            x_train, y_train, x_test, y_test = _synthetic_images((28, 28, 1), n_train, n_test, seed, signal)
            self.synthetic = True
        elif loaded is None:
            rng = np.random.default_rng(seed)
            x_train = rng.random((n_train, 28, 28, 1), dtype=np.float32)
            x_test = rng.random((n_test, 28, 28, 1), dtype=np.float32)
            y_train = _one_hot(rng.integers(0, 10, n_train), 10)
            y_test = _one_hot(rng.integers(0, 10, n_test), 10)
            self.synthetic = True
        else:
            (xt, yt), (xs, ys) = loaded
            x_train = (xt.reshape(xt.shape[0], 28, 28, 1).astype("float32") / 255)
            x_test = (xs.reshape(xs.shape[0], 28, 28, 1).astype("float32") / 255)
            y_train, y_test = _one_hot(yt, 10), _one_hot(ys, 10)
            self.synthetic = False
        super().__init__("mnist", (28, 28, 1), 10, x_train, y_train, x_test, y_test)

    @staticmethod
    def train_test_split_local(x, y):
        return train_test_split(x, y, test_size=0.1, random_state=42)

    @staticmethod
    def train_val_split_local(x, y):
        return train_test_split(x, y, test_size=0.1, random_state=42)


def _local_npz(name):
    dirs = [os.environ.get("MPLC_DATA_DIR", ""), os.path.join(os.getcwd(), "data"),
            os.path.expanduser("~/.keras/datasets")]
    for d in dirs:
        p = os.path.join(d, name) if d else ""
        if p and os.path.exists(p):
            with np.load(p, allow_pickle=False) as f:
                return (f["x_train"], f["y_train"]), (f["x_test"], f["y_test"])
    return None


class Cifar10(Dataset):
    """mplc/dataset.py:107-210 (model: the engine's batched CIFAR10 CNN, mplc/cifar.py).  Loads a local
    ``cifar10.npz`` (x_train [50000,32,32,3] uint8, y_train, x_test, y_test) from $MPLC_DATA_DIR, ./data or
    ~/.keras/datasets - the reference downloads it (mplc/dataset.py:123-150), impossible offline.  Without it,
    ``synthetic=True`` gives tensors of CIFAR10's exact shapes (x ~ U[0,1) float32, one-hot labels)."""

    def __init__(self, synthetic=None, seed=0, n_train=50000, n_test=10000, signal=0.0):
        loaded = None if synthetic else _local_npz("cifar10.npz")
        if loaded is None:
            _synthetic_allowed(synthetic, "cifar10.npz")
            x_train, y_train, x_test, y_test = _synthetic_images((32, 32, 3), n_train, n_test, seed, signal)
            self.synthetic = True
        else:
            (xt, yt), (xs, ys) = loaded
            x_train = xt.astype("float32") / 255  # preprocess_dataset_inputs, mplc/dataset.py:155-160
            x_test = xs.astype("float32") / 255
            y_train, y_test = _one_hot(np.asarray(yt).ravel(), 10), _one_hot(np.asarray(ys).ravel(), 10)
            self.synthetic = False
        super().__init__("cifar10", (32, 32, 3), 10, x_train, y_train, x_test, y_test)

    @staticmethod
    def train_test_split_local(x, y):
        return train_test_split(x, y, test_size=0.1, random_state=42)

    @staticmethod
    def train_val_split_local(x, y):
        return train_test_split(x, y, test_size=0.1, random_state=42)


class Titanic(Dataset):
    """mplc/dataset.py:212-394: 27 engineered features, binary label; model = L2 logistic regression
    (the engine's batched exact solver, mplc/lr.py).  Loads a local ``titanic.csv`` (the file the reference
    caches under mplc/local_data/titanic/) from $MPLC_DATA_DIR or ./data and applies the reference's
    feature engineering (mplc/dataset.py:235-258, including its Sex == "Male" quirk); without it, a
    Titanic-shaped synthetic set (make_classification(887, 27, n_informative=8, random_state=0))."""

    def __init__(self, synthetic=None, x=None, y=None):
        self.num_classes = 2
        if x is None:
            x, y, self.synthetic = self._load(synthetic)
        else:
            self.synthetic = False
        x = np.asarray(x, dtype=np.float32)
        y = np.asarray(y, dtype=np.float32)
        x_train, x_test, y_train, y_test = train_test_split(x, y, test_size=0.1, random_state=42)
        super().__init__("titanic", (x.shape[1],), 2, x_train, y_train, x_test, y_test)

    @staticmethod
    def _load(synthetic):
        if not synthetic:
            for d in (os.environ.get("MPLC_DATA_DIR", ""), os.path.join(os.getcwd(), "data")):
                p = os.path.join(d, "titanic.csv") if d else ""
                if p and os.path.exists(p):
                    import pandas as pd
                    raw = pd.read_csv(p)
                    if raw.columns[0].startswith("Unnamed"):
                        raw = raw.drop(raw.columns[0], axis=1)
                    xdf = raw.drop("Survived", axis=1)
                    xdf["Fam_size"] = xdf["Siblings/Spouses Aboard"] + xdf["Parents/Children Aboard"]
                    xdf["Name_Len"] = [len(i) for i in xdf["Name"]]
                    xdf["Is_alone"] = [i == 0 for i in xdf["Fam_size"]]
                    xdf["Sex"] = [i == "Male" for i in xdf["Sex"]]
                    xdf["Title"] = [i.split()[0] for i in xdf["Name"]]
                    xdf = pd.concat([xdf, pd.get_dummies(xdf["Title"])], axis=1)
                    xdf = pd.concat([xdf, pd.get_dummies(xdf["Pclass"])], axis=1)
                    xdf = xdf.drop(["Name", "Pclass", "Siblings/Spouses Aboard", "Parents/Children Aboard", "Title"],
                                   axis=1)
                    return xdf.to_numpy(dtype="float32"), raw["Survived"].to_numpy(dtype="float32"), False
        _synthetic_allowed(synthetic, "titanic.csv")
        from sklearn.datasets import make_classification
        X, y = make_classification(n_samples=887, n_features=27, n_informative=8, random_state=0)
        return X.astype("float32"), y.astype("float32"), True

    @staticmethod
    def train_test_split_local(x, y):
        return train_test_split(x, y, test_size=0.1, random_state=42)

    @staticmethod
    def train_val_split_local(x, y):
        return train_test_split(x, y, test_size=0.1, random_state=42)


class ArrayDataset(Dataset):
    """An MNIST-shaped dataset from caller arrays (tests, sklearn digits upsampled, private data).
    Uses the MNIST local splits (train_test_split 0.1, random_state 42, twice)."""

    def __init__(self, x_train, y_train, x_test, y_test, name="mnist", num_classes=10, input_shape=None):
        if input_shape is None:
            input_shape = tuple(np.asarray(x_train).shape[1:]) if name != "mnist" else (28, 28, 1)
        super().__init__(name, input_shape, num_classes, x_train, y_train, x_test, y_test)

    train_test_split_local = staticmethod(Mnist.train_test_split_local)
    train_val_split_local = staticmethod(Mnist.train_val_split_local)


def digits_as_mnist(seed=0, noise=0.02):
    """sklearn's bundled 8x8 digits (no network) upsampled x3 and padded to 28x28, values / 16, plus a
    little seeded uniform noise: a small real, learnable MNIST-shaped dataset for accuracy tests.  The noise
    breaks the exact pixel symmetries of the block upsampling (which would create exact max-pool ties whose
    winner then depends on the last bit of each implementation's conv sums).  Returns (x, y_onehot)."""
    from sklearn.datasets import load_digits
    d = load_digits()
    x = d.images.astype(np.float32) / 16.0
    x = np.kron(x, np.ones((3, 3), dtype=np.float32))
    x = np.pad(x, ((0, 0), (2, 2), (2, 2)))[..., None]
    if noise:
        x = (x * (1 - noise) + noise * np.random.default_rng(seed).random(x.shape, dtype=np.float32))
        x = x.astype(np.float32)
    y = _one_hot(d.target, 10)
    return x, y


def digits_as_cifar(seed=0, noise=0.05):
    """sklearn's digits upsampled x4 to 32x32 with three differently weighted colour channels and seeded
    uniform noise: a small, real, learnable CIFAR10-shaped dataset for accuracy tests (no network)."""
    from sklearn.datasets import load_digits
    d = load_digits()
    x = d.images.astype(np.float32) / 16.0
    x = np.kron(x, np.ones((4, 4), dtype=np.float32))
    x = np.stack([x, 0.7 * x + 0.3 * x[:, ::-1, :], 0.5 * x + 0.5 * x[:, :, ::-1]], axis=-1)
    rng = np.random.default_rng(seed)
    x = (x * (1 - noise) + noise * rng.random(x.shape, dtype=np.float32)).astype(np.float32)
    return x, _one_hot(d.target, 10)


__all__ = ["Dataset", "Mnist", "Cifar10", "Titanic", "ArrayDataset", "digits_as_mnist", "digits_as_cifar",
           "constants"]
