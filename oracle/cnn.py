"""ORACLE (test infrastructure only) - CPU restatement of the reference's MNIST-CNN coalition value.

Restates, one coalition at a time like the reference, what v(S) is:
  model      mplc/dataset.py:457-479  Conv(32,3x3,relu) Conv(64,3x3,relu) MaxPool2 Flatten Dense(128,relu)
             Dense(10,softmax); categorical CE (from logits: Keras' TF backend takes the softmax op's input,
             so dL/dz = (softmax - y)/b); Keras 2.3.1 Adam lr 1e-3, beta 0.9/0.999, eps 1e-7
  FedAvg     mplc/multi_partner_learning.py:195-216, 285-334 (fresh model per partner per round, np.average
             aggregation of mplc/mpl_utils.py:90-115, early stop :177-193)
  singleton  mplc/multi_partner_learning.py:238-269 (one fit, E epochs, persistent Adam, EarlyStopping)
  score      test accuracy (mplc/multi_partner_learning.py:158-169)
in torch-CPU float32 with autograd.  The Keras/TF arithmetic itself cannot run in this image (no TF, no
network): parity is UNPINNED at the Keras boundary and anchored on the reference tests' accuracy
thresholds.  Randomness that the reference leaves unseeded (weight init, shuffles) is defined by the
engine's keyed counters; this file restates those counters bit for bit in numpy (init_params, the
sample schedule), so engine and oracle train on identical initial weights and identical batches.
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
STRIDE = 1199936
OFF = {"W1": (0, (3, 3, 1, 32)), "b1": (288, (32,)), "W2": (320, (3, 3, 32, 64)), "b2": (18752, (64,)),
       "W3": (18816, (9216, 128)), "b3": (1198464, (128,)), "W4": (1198592, (128, 10)), "b4": (1199872, (10,))}
LIMITS = {"W1": np.float32(float.fromhex("0x1.23170ep-3")), "W2": np.float32(float.fromhex("0x1.555556p-4")),
          "W3": np.float32(float.fromhex("0x1.9f2c4cp-6")), "W4": np.float32(float.fromhex("0x1.ab099ap-3"))}
PATIENCE = 10


def mix64_np(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def mix64(z):
    return int(mix64_np(np.uint64(z & 0xFFFFFFFFFFFFFFFF)))


def subkey(key, a, b):
    return mix64(key ^ mix64(((a & 0xFFFFFFFF) << 32) | (b & 0xFFFFFFFF)))


def keyed_perm(key, n, i):
    """Vectorised restatement of keyed_perm in csrc/mnist_cnn.hip (Feistel + cycle walking)."""
    i = np.asarray(i, dtype=np.uint64)
    if n <= 1:
        return np.zeros_like(i)
    bits = int(n - 1).bit_length()
    h = (bits + 1) >> 1
    mask = np.uint64((1 << h) - 1)
    key = np.uint64(key)
    x = i.copy()
    todo = np.ones(x.shape, dtype=bool)
    out = np.zeros_like(x)
    while np.any(todo):
        L = x >> np.uint64(h)
        R = x & mask
        for rd in range(4):
            F = mix64_np(key ^ np.uint64(rd << 40) ^ R) & mask
            L, R = R, L ^ F
        x = (L << np.uint64(h)) | R
        done = todo & (x < np.uint64(n))
        out[done] = x[done]
        todo &= ~done
    return out


def init_key(seed, mask):
    return mix64(mix64(seed + 0x1517) ^ mask)


def shuffle_key(seed, mask, partner):
    return mix64(mix64(mix64(seed + 0x5EED) ^ mask) ^ (partner + 1))


def init_params(key):
    """Bit-exact restatement of init_params_kernel: glorot_uniform from mix64(key + i*golden)."""
    row = np.zeros(STRIDE, dtype=np.float32)
    i = np.arange(STRIDE, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = mix64_np(np.uint64(key) + i * np.uint64(0x9E3779B97F4A7C15))
    u = (h >> np.uint64(40)).astype(np.uint32).astype(np.float32) * np.float32(2.0 ** -24)
    w = (u * np.float32(2.0) - np.float32(1.0))
    for name, lim in LIMITS.items():
        off, shape = OFF[name]
        n = int(np.prod(shape))
        row[off:off + n] = w[off:off + n] * lim
    return row


def seq_order_key(seed, mask):
    return mix64(mix64(seed + 0x5E90) ^ mask)


def seq_member_order(seed, mask, k, e, m):
    """Member indices (ascending-partner positions) of a sequential coalition's round (e, m), in the order
    they train (csrc/keyed.h seq_locate; the reference draws np.random.permutation, :365)."""
    okey = subkey(seq_order_key(seed, mask), 0x60000 + e, m)
    return [int(v) for v in keyed_perm(okey, k, np.arange(k))]


def minibatch_bounds(n, M):
    split_indices = np.arange(1, M + 1) / M
    return [0] + [int(v) for v in (split_indices[:-1] * n).astype(int)] + [int(n)]


def fedavg_round_rows(key, rows, bs, M, e, m):
    """Row indices of each Keras step of partner `rows` in round m of epoch e (FedAvg replica)."""
    n = len(rows)
    b = minibatch_bounds(n, M)
    s0, s1 = b[m], b[m + 1]
    L = s1 - s0
    q = keyed_perm(subkey(key, 0x20000 + e, m), L, np.arange(L))
    pos = keyed_perm(subkey(key, 0x10000 + e, 0), n, np.uint64(s0) + q)
    order = np.asarray(rows)[pos.astype(np.int64)]
    return [order[t:t + bs] for t in range(0, L, bs)]


def single_epoch_rows(key, rows, bs, e):
    n = len(rows)
    pos = keyed_perm(subkey(key, 0x30000 + e, 0), n, np.arange(n))
    order = np.asarray(rows)[pos.astype(np.int64)]
    return [order[t:t + bs] for t in range(0, n, bs)]


# ------------------------------------------------------------------------------------------------
# torch-CPU model
# ------------------------------------------------------------------------------------------------
def _torch():
    import torch
    torch.set_num_threads(max(1, torch.get_num_threads()))
    return torch


def unpack(row):
    torch = _torch()
    out = {}
    for name, (off, shape) in OFF.items():
        n = int(np.prod(shape))
        out[name] = torch.from_numpy(np.array(row[off:off + n], dtype=np.float32).reshape(shape))
    return out


def pack(p):
    row = np.zeros(STRIDE, dtype=np.float32)
    for name, (off, shape) in OFF.items():
        row[off:off + int(np.prod(shape))] = p[name].detach().numpy().reshape(-1)
    return row


def forward(p, x):
    """x: [b,28,28] float32 tensor -> logits [b,10] (NHWC flatten order, as Keras)."""
    torch = _torch()
    F = torch.nn.functional
    h = x.unsqueeze(1)
    h = F.relu(F.conv2d(h, p["W1"].permute(3, 2, 0, 1), p["b1"]))
    h = F.relu(F.conv2d(h, p["W2"].permute(3, 2, 0, 1), p["b2"]))
    h = F.max_pool2d(h, 2)
    h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)
    h = F.relu(h @ p["W3"] + p["b3"])
    return h @ p["W4"] + p["b4"]


def gradients(p, x, y, dtype=None):
    """Autograd gradients of the batch-mean CE; dtype=torch.float64 gives the high-precision reference."""
    torch = _torch()
    if dtype is not None:
        p = {k: v.to(dtype) for k, v in p.items()}
        x = x.to(dtype)
    q = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    logits = forward(q, x)
    loss = torch.nn.functional.cross_entropy(logits, y)  # mean over batch, from logits
    loss.backward()
    return {k: v.grad.detach() for k, v in q.items()}, float(loss.detach())


def conv1_relu_flip_bound(p, x, y, rel_tau=1e-6):
    """Upper bound on how much the W1 / b1 gradients can move if the ReLU mask of conv1 flips at positions
    whose pre-activation is within rel_tau * max|a1| of zero (fp32 recomputations in a different summation
    order may land on either side): |pix| * |dL/da1| summed over those positions, in fp64."""
    torch = _torch()
    F = torch.nn.functional
    p = {k: v.to(torch.float64) for k, v in p.items()}
    x = x.to(torch.float64)
    z1 = F.conv2d(x.unsqueeze(1), p["W1"].permute(3, 2, 0, 1), p["b1"])
    a1 = F.relu(z1).detach().requires_grad_(True)
    h = F.max_pool2d(F.relu(F.conv2d(a1, p["W2"].permute(3, 2, 0, 1), p["b2"])), 2)
    h = F.relu(h.permute(0, 2, 3, 1).reshape(h.shape[0], -1) @ p["W3"] + p["b3"])
    loss = F.cross_entropy(h @ p["W4"] + p["b4"], y)
    loss.backward()
    da1 = a1.grad.abs()                                   # [b, 32, 26, 26]
    az = z1.detach().abs()
    near = ((az > 0) & (az <= rel_tau * az.max())).to(torch.float64)  # exact zeros agree on both sides
    w = da1 * near
    patches = F.unfold(x.unsqueeze(1).abs(), 3)           # [b, 9, 676]
    bw = torch.einsum("bkp,bcp->kc", patches, w.reshape(w.shape[0], 32, -1))
    return bw.reshape(-1).numpy(), w.sum(dim=(0, 2, 3)).numpy()


class KerasAdam:
    """Keras 2.3.1 Adam (keras/optimizers.py get_updates), float32."""

    def __init__(self, params, lr=0.001, beta_1=0.9, beta_2=0.999, eps=1e-7, precise=False):
        """precise=True: the same fp32 constants, every derived scalar kept in fp64 (with fp64 params: the
        high-precision restatement of the same update)."""
        torch = _torch()
        self.lr, self.b1, self.b2, self.eps = (np.float32(lr), np.float32(beta_1), np.float32(beta_2), np.float32(eps))
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}
        self.t = 0
        self.precise = precise

    def step(self, params, grads):
        torch = _torch()
        self.t += 1
        if self.precise:
            b1, b2 = float(self.b1), float(self.b2)
            lr_t = float(self.lr) * np.sqrt(1.0 - b2 ** self.t) / (1.0 - b1 ** self.t)
            for k in params:
                g = grads[k]
                self.m[k] = b1 * self.m[k] + (1.0 - b1) * g
                self.v[k] = b2 * self.v[k] + (1.0 - b2) * (g * g)
                params[k] = params[k] - lr_t * self.m[k] / (torch.sqrt(self.v[k]) + float(self.eps))
            return
        t = np.float32(self.t)
        lr_t = self.lr * (np.sqrt(np.float32(1) - np.power(self.b2, t)) / (np.float32(1) - np.power(self.b1, t)))
        lr_t = float(np.float32(lr_t))
        for k in params:
            g = grads[k]
            self.m[k] = float(self.b1) * self.m[k] + float(np.float32(1) - self.b1) * g
            self.v[k] = float(self.b2) * self.v[k] + float(np.float32(1) - self.b2) * (g * g)
            params[k] = params[k] - lr_t * self.m[k] / (torch.sqrt(self.v[k]) + float(self.eps))


def evaluate(p, x, y, batch=1000):
    """[mean CE, accuracy] like Keras evaluate (mplc/multi_partner_learning.py:142-169)."""
    torch = _torch()
    correct, loss = 0, 0.0
    dt = p["W1"].dtype  # fp64 parameters (precise runs) evaluate in fp64
    with torch.no_grad():
        for s in range(0, len(y), batch):
            z = forward(p, x[s:s + batch].to(dt))
            loss += float(torch.nn.functional.cross_entropy(z, y[s:s + batch], reduction="sum"))
            correct += int((z.argmax(1) == y[s:s + batch]).sum())
    return loss / len(y), correct / len(y)


class Data:
    def __init__(self, x_train, y_train, x_val, y_val, x_test, y_test):
        torch = _torch()

        def lab(y):
            y = np.asarray(y)
            return torch.from_numpy((np.argmax(y, 1) if y.ndim == 2 else y).astype(np.int64))

        def img(x):
            x = np.asarray(x, dtype=np.float32)
            return torch.from_numpy(np.ascontiguousarray(x.reshape(x.shape[0], 28, 28)))
        self.x_train, self.y_train = img(x_train), lab(y_train)
        self.x_val, self.y_val = img(x_val), lab(y_val)
        self.x_test, self.y_test = img(x_test), lab(y_test)


def average_models(glob, models, w, keep_f64=False):
    """np.average(..., axis=0, weights=w) per layer in float64 -> float32 (mplc/mpl_utils.py:90-102);
    keep_f64: the float64 average itself (the fp64 restatement)."""
    torch = _torch()
    new = {}
    for k in glob:
        stack = np.array([pm[k].numpy() for pm in models])
        avg = np.average(stack, axis=0, weights=w)
        new[k] = torch.from_numpy(avg if keep_f64 else avg.astype(np.float32))
    return new


def fedavg_round(data, partner_rows, batch_sizes, coalition, glob, seed=0, M=20, e=0, m=0, precise=False):
    """One FedAvg round (epoch e, minibatch m; mplc/multi_partner_learning.py:301-334) from the global model
    `glob` (dict of tensors): every partner a fresh Keras Adam over its round rows at its batch size, then the
    data-volume average (mplc/mpl_utils.py:90-115).  precise=True runs the same schedule with every tensor
    operation in float64 (gradients, Adam, the average kept in fp64): the high-precision reference of the same
    algorithm against which fp32 implementations' rounding is measured."""
    torch = _torch()
    coalition = tuple(sorted(coalition))
    mask = sum(1 << p for p in coalition)
    dt = torch.float64 if precise else torch.float32
    sizes = [len(partner_rows[p]) for p in coalition]
    w = np.asarray(sizes) / np.sum(sizes)
    models = []
    for p_id in coalition:
        key = shuffle_key(seed, mask, p_id)
        params = {k: v.to(dt).clone() for k, v in glob.items()}
        opt = KerasAdam(params, precise=precise)
        for rows in fedavg_round_rows(key, partner_rows[p_id], batch_sizes[p_id], M, e, m):
            g, _ = gradients(params, data.x_train[rows], data.y_train[rows], dtype=dt if precise else None)
            opt.step(params, g)
        models.append(params)
    return average_models(glob, models, w, keep_f64=precise)


class _FitLog:
    """Keras fit history of one fit: running training CE / accuracy over the fit's batches (each batch's
    values before its update, sample-weighted), then val metrics of the fitted model
    (mplc/multi_partner_learning.py:130-133 log_partner_perf; mplc/mpl_utils.py:11-27)."""

    def __init__(self):
        self.loss, self.correct, self.n = 0.0, 0, 0

    def batch(self, params, x, y, loss_mean):
        torch = _torch()
        with torch.no_grad():
            self.correct += int((forward(params, x).argmax(1) == y).sum())
        self.loss += loss_mean * len(y)
        self.n += len(y)

    def store(self, h, e, m, params, data):
        vl, va = evaluate(params, data.x_val, data.y_val)
        h["val_loss"][e, m], h["val_accuracy"][e, m] = vl, va
        h["loss"][e, m] = self.loss / self.n if self.n else np.nan
        h["accuracy"][e, m] = self.correct / self.n if self.n else np.nan


HISTORY_METRICS = ("val_accuracy", "val_loss", "loss", "accuracy")


def coalition_value(data, partner_rows, batch_sizes, coalition, seed=0, epochs=1, M=10,
                    aggregation="data-volume", early_stopping=False, return_model=False, approach="fedavg",
                    history=None, es_trace=None, precise=False):
    """v(S) of one coalition, the reference's way (sequential), on the engine's keyed init and order.
    With a `history` dict, the learning history (mplc/mpl_utils.py:11-27) is recorded into it; with an
    `es_trace` list, the val losses the early-stopping rule compares are appended to it.  precise=True (FedAvg
    and singletons): the same schedule and fp32 constants with every tensor operation in float64 - gradients,
    Adam, the average (kept in fp64) and the test evaluation: the high-precision value of the same algorithm."""
    torch = _torch()
    coalition = tuple(sorted(coalition))
    mask = sum(1 << p for p in coalition)
    glob = unpack(init_params(init_key(seed, mask)))
    dt = torch.float64 if precise else None
    if precise:
        if approach != "fedavg" or history is not None:
            raise ValueError("precise=True restates FedAvg / singleton training without history")
        glob = {k: v.to(dt) for k, v in glob.items()}
    epochs_done = epochs
    if history is not None:
        for p_id in coalition:
            history[p_id] = {k: np.full((epochs, M), np.nan) for k in HISTORY_METRICS}
        if len(coalition) > 1:
            history["mpl_model"] = {"val_accuracy": np.zeros((epochs, M)), "val_loss": np.zeros((epochs, M))}
    if len(coalition) == 1:
        p_id = coalition[0]
        key = shuffle_key(seed, mask, p_id)
        params = {k: v.clone() for k, v in glob.items()}
        opt = KerasAdam(params, precise=precise)
        best, wait = np.inf, 0
        log = None
        for e in range(epochs):
            log = _FitLog() if history is not None else None
            for rows in single_epoch_rows(key, partner_rows[p_id], batch_sizes[p_id], e):
                g, lm = gradients(params, data.x_train[rows], data.y_train[rows], dtype=dt)
                if log is not None:
                    log.batch(params, data.x_train[rows], data.y_train[rows], lm)
                opt.step(params, g)
            if early_stopping and epochs > PATIENCE:
                vl, _ = evaluate(params, data.x_val, data.y_val)
                if es_trace is not None:
                    es_trace.append(vl)
                if vl < best:
                    best, wait = vl, 0
                else:
                    wait += 1
                    if wait >= PATIENCE:
                        epochs_done = e + 1
                        break
        glob = params
        if log is not None:  # SinglePartnerLearning logs the last epoch at [0, 0]
            log.store(history[p_id], 0, 0, params, data)
    else:
        sizes = [len(partner_rows[p]) for p in coalition]
        if aggregation == "uniform":
            w = [1 / len(coalition)] * len(coalition)
        else:
            w = np.asarray(sizes) / np.sum(sizes)
        val_hist = []
        for e in range(epochs):
            if early_stopping and epochs > PATIENCE:
                val_hist.append(evaluate(glob, data.x_val, data.y_val)[0])
                if es_trace is not None:
                    es_trace.append(val_hist[-1])
            for m in range(M):
                if history is not None:  # round-start collective model (eval_and_log_model_val_perf)
                    vl, va = evaluate(glob, data.x_val, data.y_val)
                    history["mpl_model"]["val_loss"][e, m], history["mpl_model"]["val_accuracy"][e, m] = vl, va
                if approach != "fedavg":
                    # seq-pure / seq-with-final-agg / seqavg (mplc/multi_partner_learning.py:337-433): one model
                    # and one optimizer per round, members in the round's shuffled order, snapshots per member
                    params = {k: v.clone() for k, v in glob.items()}
                    opt = KerasAdam(params)
                    snaps = [None] * len(coalition)
                    for mi in seq_member_order(seed, mask, len(coalition), e, m):
                        p_id = coalition[mi]
                        key = shuffle_key(seed, mask, p_id)
                        log = _FitLog() if history is not None else None
                        for rows in fedavg_round_rows(key, partner_rows[p_id], batch_sizes[p_id], M, e, m):
                            g, lm = gradients(params, data.x_train[rows], data.y_train[rows])
                            if log is not None:
                                log.batch(params, data.x_train[rows], data.y_train[rows], lm)
                            opt.step(params, g)
                        snaps[mi] = {k: v.clone() for k, v in params.items()}
                        if log is not None:
                            log.store(history[p_id], e, m, params, data)
                    if approach == "seqavg" or (approach == "seq-with-final-agg" and m == M - 1):
                        glob = average_models(glob, snaps, w)
                    else:
                        glob = params
                    continue
                partner_models = []
                for p_id in coalition:
                    key = shuffle_key(seed, mask, p_id)
                    params = {k: v.clone() for k, v in glob.items()}
                    opt = KerasAdam(params, precise=precise)  # fresh optimizer per partner fit
                    log = _FitLog() if history is not None else None
                    for rows in fedavg_round_rows(key, partner_rows[p_id], batch_sizes[p_id], M, e, m):
                        g, lm = gradients(params, data.x_train[rows], data.y_train[rows], dtype=dt)
                        if log is not None:
                            log.batch(params, data.x_train[rows], data.y_train[rows], lm)
                        opt.step(params, g)
                    if log is not None:
                        log.store(history[p_id], e, m, params, data)
                    partner_models.append(params)
                glob = average_models(glob, partner_models, w, keep_f64=precise)
            if early_stopping and epochs > PATIENCE and e >= PATIENCE and val_hist[e] > val_hist[e - PATIENCE]:
                epochs_done = e + 1
                break
    _, acc = evaluate(glob, data.x_test, data.y_test)
    if return_model:  # a model row; precise runs return the fp64 tensors themselves
        return acc, epochs_done, ({k: v.detach().clone() for k, v in glob.items()} if precise else pack(glob))
    return acc, epochs_done
