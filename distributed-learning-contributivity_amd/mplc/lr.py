"""Titanic logistic-regression coalition engine (host side of csrc/logreg.hip).

All requested coalitions are trained in ONE launch (a workgroup per coalition runs its whole FedAvg:
epochs x minibatch rounds x partner fits + aggregation + test accuracy).  See include/mplc_hip.h
``mplc_lr_fedavg`` for the semantics and the reference lines it replaces.
"""
import numpy as np

from . import _native
from .cnn import minibatch_bounds, shuffle_key
from .fedavg import aggregation_weights

MAXP = 64


def _mix64_np(z):
    """cnn.mix64 on a uint64 array (numpy's uint64 products wrap mod 2^64, the & M64 of the scalar form)."""
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def coalition_tables(coalitions, partner_sizes, seed, aggregation):
    """The launch's per-coalition tables, vectorised over coalitions: bit masks, each member's shuffle key
    (cnn.shuffle_key), the np.average weights and scale of aggregation_weights.  Equal, element for element, to
    the per-coalition loop (tests/test_lr.py); the loop cost about 35 ms per 1023-coalition sweep on the host."""
    C = len(coalitions)
    n = len(partner_sizes)
    lens = np.fromiter((len(c) for c in coalitions), dtype=np.int64, count=C)
    flat = np.fromiter((p for c in coalitions for p in c), dtype=np.int64, count=int(lens.sum()))
    if np.any(lens > MAXP) or (len(flat) and (flat.min() < 0 or flat.max() >= n)):
        raise ValueError("invalid coalition: more than 64 partners or a partner id out of range")
    member = np.zeros((C, n), dtype=bool)
    member[np.repeat(np.arange(C), lens), flat] = True
    bits = np.left_shift(np.uint64(1), np.arange(n, dtype=np.uint64))
    masks = (member * bits).sum(axis=1, dtype=np.uint64)
    counts = member.sum(axis=1)
    # member i of a coalition = the i-th set bit: its partner id
    order = np.argsort(~member, axis=1, kind="stable")[:, :min(n, MAXP)]
    slot = np.arange(order.shape[1])[None, :] < counts[:, None]
    with np.errstate(over="ignore"):
        base = _mix64_np(np.full(C, _mix64_np(np.array([(seed + 0x5EED) & ((1 << 64) - 1)], dtype=np.uint64))[0],
                                 dtype=np.uint64) ^ masks)
        k = _mix64_np(base[:, None] ^ (order.astype(np.uint64) + np.uint64(1)))
    keys = np.zeros((C, MAXP), dtype=np.uint64)
    keys[:, :order.shape[1]] = np.where(slot, k, np.uint64(0))
    w = np.zeros((C, MAXP), dtype=np.float64)
    scale = np.ones(C, dtype=np.float64)
    sizes = np.asarray(partner_sizes)
    for P in np.unique(counts):  # one vectorised aggregation_weights per coalition size (same reductions)
        if P < 2:
            continue
        sel = np.nonzero(counts == P)[0]
        sz = sizes[order[sel, :P]]
        if aggregation == "uniform":
            ww = np.full((len(sel), P), 1 / P)
        elif aggregation == "data-volume":
            ww = sz / np.sum(sz, axis=1, keepdims=True)
        else:
            raise ValueError(f"aggregation approach '{aggregation}' is not a valid approach. ")
        scl = ww.sum(axis=1)
        if np.any(scl == 0.0):
            raise ZeroDivisionError("Weights sum to zero, can't be normalized")
        w[sel, :P] = ww
        scale[sel] = scl
    return masks, keys, w, scale


class LogRegEngine:
    def __init__(self, *, x_train, y_train, x_val, y_val, x_test, y_test, partner_rows, epoch_count, minibatch_count,
                 aggregation="data-volume", is_early_stopping=True, seed=0, device=None, **_):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("MI355X (HIP) device required: the MPLC engine has no CPU fallback")
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.seed = int(seed)
        self.epoch_count = int(epoch_count)
        self.minibatch_count = int(minibatch_count)
        self.aggregation = aggregation
        self.is_early_stopping = bool(is_early_stopping)

        def feats(x):
            return torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=np.float32))).to(self.device)

        def labs(y):
            y = np.asarray(y)
            if y.ndim == 2:
                y = np.argmax(y, axis=1)
            return torch.from_numpy(np.ascontiguousarray(y.astype(np.float32))).to(self.device)

        self.x_train_d, self.y_train_d = feats(x_train), labs(y_train)
        self.x_val_d, self.y_val_d = feats(x_val), labs(y_val)
        self.x_test_d, self.y_test_d = feats(x_test), labs(y_test)
        self.n_features = int(self.x_train_d.shape[1])
        self.partner_sizes = [int(len(r)) for r in partner_rows]
        rows, offs, splits = [], [], []
        for r in partner_rows:
            offs.append(len(rows))
            rows.extend(int(i) for i in r)
            splits.extend(minibatch_bounds(len(r), self.minibatch_count))
        i32 = dict(dtype=torch.int32, device=self.device)
        self.rows_d = torch.tensor(rows, **i32)
        self.rows_off_d = torch.tensor(offs, **i32)
        self.n_rows_d = torch.tensor(self.partner_sizes, **i32)
        self.splits_d = torch.tensor(splits, **i32)
        self.stats = {"coalitions": 0, "batches": 0, "replicas": 0}
        self.profiler = None
        self.last_theta = None

    supports_history = True
    HIST_BLOCK = 2 + 4 * MAXP
    # coalitions per mplc_lr_fedavg call: its stream-ordered workspace holds every coalition's partner fits (C x 64 x
    # 32 doubles, 16 KB per coalition), so an exact sweep over 2^20 coalitions would ask for ~17 GB at once (ADVICE
    # r5); each coalition's fits are independent of the others in the call, so chunks give the same values
    CALL_COALITIONS = 32768

    def evaluate(self, coalitions, epoch_count=None, is_early_stopping=None, return_details=False,
                 record_history=False, return_models=False):
        """v(S) for each coalition; with record_history (one coalition) the details also hold its learning
        history (mplc/mpl_utils.py:11-27) in the layout of multi_partner_learning.History."""
        coalitions = [tuple(sorted(int(i) for i in c)) for c in coalitions]
        if len(coalitions) > self.CALL_COALITIONS:
            if record_history:
                raise ValueError("record_history takes exactly one coalition")
            scores, epochs, thetas = [], [], []
            for i in range(0, len(coalitions), self.CALL_COALITIONS):
                scores.append(self._evaluate_call(coalitions[i:i + self.CALL_COALITIONS], epoch_count,
                                                  is_early_stopping, False, False, False))
                epochs.append(self.last_epochs_done)
                thetas.append(self.last_theta)
            scores = np.concatenate(scores)
            self.last_epochs_done, self.last_theta = np.concatenate(epochs), np.concatenate(thetas)
            if not return_details:
                return scores
            out = {"scores": scores, "epochs_done": self.last_epochs_done}
            if return_models:
                out["models"] = [self.last_theta[ci].reshape(1, -1).copy() for ci in range(len(coalitions))]
            return out
        return self._evaluate_call(coalitions, epoch_count, is_early_stopping, return_details, record_history,
                                   return_models)

    def _evaluate_call(self, coalitions, epoch_count, is_early_stopping, return_details, record_history,
                       return_models):
        import torch
        C = len(coalitions)
        if record_history and C != 1:
            raise ValueError("record_history takes exactly one coalition")
        E = self.epoch_count if epoch_count is None else int(epoch_count)
        es = self.is_early_stopping if is_early_stopping is None else bool(is_early_stopping)
        masks, keys, w, scale = coalition_tables(coalitions, self.partner_sizes, self.seed, self.aggregation)
        dev = self.device
        t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        masks_d = t(masks.view(np.int64))
        keys_d = t(keys.view(np.int64).reshape(-1).copy())
        w_d, scale_d = t(w.reshape(-1).copy()), t(scale)
        correct = torch.zeros(C, dtype=torch.int32, device=dev)
        epochs_done = torch.zeros(C, dtype=torch.int32, device=dev)
        theta = torch.zeros((C, self.n_features + 1), dtype=torch.float64, device=dev)
        M = self.minibatch_count
        hist, stride = None, 0
        if record_history:  # partner entries NaN, collective entries 0 until logged (History.__init__)
            stride = E * M * self.HIST_BLOCK
            h0 = np.zeros((E, M, self.HIST_BLOCK))
            h0[:, :, 2:] = np.nan
            hist = torch.from_numpy(h0.reshape(-1)).to(dev)
        P = _native.ptr
        st = _native.lib().mplc_lr_fedavg(
            P(self.x_train_d), P(self.y_train_d), self.n_features, P(self.rows_d), P(self.rows_off_d), P(self.n_rows_d),
            P(self.splits_d), self.minibatch_count, P(masks_d), P(keys_d), P(w_d), P(scale_d), C, E, 1 if es else 0,
            P(self.x_val_d), P(self.y_val_d), int(self.y_val_d.numel()), P(self.x_test_d), P(self.y_test_d),
            int(self.y_test_d.numel()), P(correct), P(epochs_done), P(theta),
            P(hist) if hist is not None else None, stride, _native.stream_handle(dev))
        _native.check(st, "mplc_lr_fedavg")
        scores = correct.cpu().numpy().astype(np.float64) / float(self.y_test_d.numel())
        self.last_theta = theta.cpu().numpy()
        self.last_epochs_done = epochs_done.cpu().numpy().astype(np.int64)  # realised epochs (early stopping)
        self.stats["coalitions"] += C
        self.stats["batches"] += 1
        self.stats["replicas"] += sum(len(c) for c in coalitions)
        if return_details:
            out = {"scores": scores, "epochs_done": self.last_epochs_done}
            if return_models:  # Titanic.LogisticRegression.get_weights(): [coef | intercept], shape (1, 28)
                out["models"] = [self.last_theta[ci].reshape(1, -1).copy() for ci in range(C)]
            if hist is not None:
                out["history"] = self._history(coalitions[0], hist.cpu().numpy().reshape(E, M, self.HIST_BLOCK))
            return out
        return scores

    @staticmethod
    def _history(coal, h):
        names = ("loss", "accuracy", "val_loss", "val_accuracy")
        out = {}
        for pi, p in enumerate(coal):
            out[p] = {k: np.ascontiguousarray(h[:, :, 2 + 4 * pi + i]) for i, k in enumerate(names)}
            out[p] = {k: out[p][k] for k in ("val_accuracy", "val_loss", "loss", "accuracy")}
        if len(coal) > 1:
            out["mpl_model"] = {"val_accuracy": np.ascontiguousarray(h[:, :, 1]),
                                "val_loss": np.ascontiguousarray(h[:, :, 0])}
        return out
