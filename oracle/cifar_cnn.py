"""ORACLE (test infrastructure only) - CPU restatement of the reference's CIFAR10-CNN coalition value.

Restates, one coalition at a time like the reference, what v(S) is for the CIFAR10 model:
  model      mplc/dataset.py:167-200  Conv(32,same) ReLU Conv(32) ReLU MaxPool2 Dropout(.25) Conv(64,same) ReLU
             Conv(64) ReLU MaxPool2 Dropout(.25) Flatten Dense(512) ReLU Dropout(.5) Dense(10) softmax;
             categorical CE from logits (Keras' TF backend takes the softmax op's input); Keras 2.3.1 RMSprop
             (learning_rate 1e-4, rho 0.9, epsilon 1e-7, decay 1e-6: lr_t = lr / (1 + decay * iterations),
             iterations counted before the update); tf.nn.dropout: (x * (1/(1-rate))) * (u >= rate)
  FedAvg     mplc/multi_partner_learning.py:195-216, 285-334 (fresh model AND fresh optimizer per partner fit,
             np.average aggregation, early stop); singleton :238-269 (persistent optimizer)
  score      test accuracy, inference mode (no dropout)
in torch-CPU float32 with autograd.  TF/Keras cannot run here: parity is UNPINNED at the Keras boundary
(as for MNIST, see oracle/cnn.py).  Randomness the reference leaves unseeded (init, shuffles, dropout masks)
is defined by the engine's keyed counters; this file restates them bit for bit (init_params, the sample
schedule of oracle/cnn.py, dropout_keep).
"""
import numpy as np

from . import cnn as ocnn

STRIDE = 1251008
OFF = {"W1": (0, (3, 3, 3, 32)), "b1": (896, (32,)), "W2": (960, (3, 3, 32, 32)), "b2": (10176, (32,)),
       "W3": (10240, (3, 3, 32, 64)), "b3": (28672, (64,)), "W4": (28736, (3, 3, 64, 64)), "b4": (65600, (64,)),
       "W5": (65664, (2304, 512)), "b5": (1245312, (512,)), "W6": (1245824, (512, 10)), "b6": (1250944, (10,))}
# glorot_uniform limits sqrt(6 / (fan_in + fan_out)) rounded to fp32 (as csrc/cifar_cnn.hip)
LIMITS = {k: np.float32(float.fromhex(v)) for k, v in {
    "W1": "0x1.1aa69ep-3", "W2": "0x1.a20bd8p-4", "W3": "0x1.555556p-4", "W4": "0x1.279a74p-4",
    "W5": "0x1.7a2316p-5", "W6": "0x1.b72326p-4"}.items()}
DROP = {"L2": (2, 1 << 22), "L4": (4, 1 << 22), "L5": (5, 1 << 23)}  # layer id, threshold on the 24-bit u
SCALE_25 = np.float32(1.0) / np.float32(0.75)
PATIENCE = 10


def init_params(key):
    row = np.zeros(STRIDE, dtype=np.float32)
    i = np.arange(STRIDE, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = ocnn.mix64_np(np.uint64(key) + i * np.uint64(0x9E3779B97F4A7C15))
    u = (h >> np.uint64(40)).astype(np.uint32).astype(np.float32) * np.float32(2.0 ** -24)
    w = u * np.float32(2.0) - np.float32(1.0)
    for name, lim in LIMITS.items():
        off, shape = OFF[name]
        n = int(np.prod(shape))
        row[off:off + n] = w[off:off + n] * lim
    return row


def fedavg_drop_key(key, e, m, t):
    return ocnn.subkey(key, 0x40000 + e, (m << 16) | t)


def single_drop_key(key, e, t):
    return ocnn.subkey(key, 0x50000 + e, t)


def hash32(x):
    """lowbias32 finaliser on uint32 arrays (csrc/cifar_cnn.hip hash32)."""
    x = np.asarray(x, dtype=np.uint32)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7feb352d)
        x = x ^ (x >> np.uint32(15))
        x = x * np.uint32(0x846ca68b)
        x = x ^ (x >> np.uint32(16))
    return x


def dropout_keep(dkey, layer, count, n):
    """[count, n] bool keep mask of one layer at one step (slot j = row, element e = NHWC flat index):
    hash32(row_seed(j) ^ e) >> 8 >= rate * 2^24, row_seed = hash32(lo(key) ^ hash32(hi(key) ^ layer<<24 ^ j))."""
    lid, thr = DROP[layer]
    dkey = int(dkey)
    j = np.arange(count, dtype=np.uint32)
    inner = hash32(np.uint32(dkey >> 32) ^ np.uint32(lid << 24) ^ j)
    seed = hash32(np.uint32(dkey & 0xFFFFFFFF) ^ inner)[:, None]
    e = np.arange(n, dtype=np.uint32)[None, :]
    return (hash32(seed ^ e) >> np.uint32(8)) >= np.uint32(thr)


def step_masks(dkey, count):
    """Dropout keep masks of one training step (as float32 0/1 torch tensors in NHWC layer shapes)."""
    import torch
    return {"L2": torch.from_numpy(dropout_keep(dkey, "L2", count, 7200).reshape(count, 15, 15, 32).astype(np.float32)),
            "L4": torch.from_numpy(dropout_keep(dkey, "L4", count, 2304).reshape(count, 6, 6, 64).astype(np.float32)),
            "L5": torch.from_numpy(dropout_keep(dkey, "L5", count, 512).astype(np.float32))}


def _torch():
    import torch
    return torch


def unpack(row):
    torch = _torch()
    return {name: torch.from_numpy(np.array(row[off:off + int(np.prod(shape))], dtype=np.float32).reshape(shape))
            for name, (off, shape) in OFF.items()}


def pack(p):
    row = np.zeros(STRIDE, dtype=np.float32)
    for name, (off, shape) in OFF.items():
        row[off:off + int(np.prod(shape))] = p[name].detach().numpy().reshape(-1)
    return row


def _dropout(h_nhwc, keep, rate):
    """tf.nn.dropout: (x * scale) * keep, scale = fp32(1 / (1 - rate))."""
    torch = _torch()
    scale = float(np.float32(1.0) / np.float32(1.0 - rate)) if h_nhwc.dtype == torch.float32 else 1.0 / (1.0 - rate)
    return (h_nhwc * scale) * keep.to(h_nhwc.dtype)


def forward(p, x, masks=None, return_acts=False):
    """x: [b,32,32,3] (NHWC) -> logits [b,10].  masks None = inference (no dropout)."""
    torch = _torch()
    F = torch.nn.functional

    def conv(h, W, b, pad):
        return F.conv2d(h, W.permute(3, 2, 0, 1), b, padding=pad)

    h = x.permute(0, 3, 1, 2)
    a1 = F.relu(conv(h, p["W1"], p["b1"], 1))
    a2 = F.relu(conv(a1, p["W2"], p["b2"], 0))
    p2 = F.max_pool2d(a2, 2).permute(0, 2, 3, 1)               # NHWC [b,15,15,32]
    d2 = _dropout(p2, masks["L2"], 0.25) if masks is not None else p2
    a3 = F.relu(conv(d2.permute(0, 3, 1, 2), p["W3"], p["b3"], 1))
    a4 = F.relu(conv(a3, p["W4"], p["b4"], 0))
    p4 = F.max_pool2d(a4, 2).permute(0, 2, 3, 1)               # [b,6,6,64]
    d4 = _dropout(p4, masks["L4"], 0.25) if masks is not None else p4
    flat = d4.reshape(d4.shape[0], -1)
    h5 = F.relu(flat @ p["W5"] + p["b5"])
    d5 = _dropout(h5, masks["L5"], 0.5) if masks is not None else h5
    logits = d5 @ p["W6"] + p["b6"]
    if return_acts:
        return logits, {"a1": a1.permute(0, 2, 3, 1), "d2": d2, "a3": a3.permute(0, 2, 3, 1), "d4": flat, "d5": d5}
    return logits


def gradients(p, x, y, masks, dtype=None):
    """Autograd gradients of the batch-mean CE; dtype=torch.float64 gives the high-precision reference."""
    torch = _torch()
    if dtype is not None:
        p = {k: v.to(dtype) for k, v in p.items()}
        x = x.to(dtype)
    q = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    loss = torch.nn.functional.cross_entropy(forward(q, x, masks), y)
    loss.backward()
    return {k: v.grad.detach() for k, v in q.items()}, float(loss.detach())


class KerasRMSprop:
    """Keras 2.3.1 RMSprop (keras/optimizers.py get_updates), float32."""

    def __init__(self, params, lr=1e-4, rho=0.9, eps=1e-7, decay=1e-6, precise=False):
        """precise=True: the same fp32 constants, the decayed learning rate kept in fp64 (with fp64 params:
        the high-precision restatement of the same update)."""
        torch = _torch()
        self.lr, self.rho, self.eps, self.decay = np.float32(lr), np.float32(rho), np.float32(eps), np.float32(decay)
        self.omr = np.float32(1.0 - rho)  # (1. - self.rho) on the Python double, then fp32
        self.a = {k: torch.zeros_like(v) for k, v in params.items()}
        self.iterations = 0
        self.precise = precise

    def step(self, params, grads):
        torch = _torch()
        it = np.float32(self.iterations)
        if self.precise:
            lr_t = float(self.lr) / (1.0 + float(self.decay) * self.iterations)
        else:
            lr_t = float(self.lr * (np.float32(1.0) / (np.float32(1.0) + self.decay * it)))
        self.iterations += 1
        for k in params:
            g = grads[k]
            self.a[k] = float(self.rho) * self.a[k] + float(self.omr) * (g * g)
            params[k] = params[k] - lr_t * g / (torch.sqrt(self.a[k]) + float(self.eps))


def fedavg_round(data, partner_rows, batch_sizes, coalition, glob, seed=0, M=20, e=0, m=0, precise=False):
    """One FedAvg round of the CIFAR10 model from the global model `glob` (as oracle/cnn.py fedavg_round): each
    partner a fresh Keras RMSprop over its round rows with the step's keyed dropout masks, then the data-volume
    average.  precise=True: every tensor operation in float64 (same masks, schedule and constants)."""
    coalition = tuple(sorted(coalition))
    sizes = [len(partner_rows[p]) for p in coalition]
    w = np.asarray(sizes) / np.sum(sizes)
    models = partner_fits(data, partner_rows, batch_sizes, coalition, glob, seed, M, e, m, precise)
    return ocnn.average_models(glob, models, w, keep_f64=precise)


def partner_fits(data, partner_rows, batch_sizes, coalition, glob, seed=0, M=20, e=0, m=0, precise=False):
    """The partner models of one FedAvg round before the average (fedavg_round), in sorted coalition order
    (multi_partner_learning.py:301-334: each partner fits a fresh model from the global weights)."""
    torch = _torch()
    coalition = tuple(sorted(coalition))
    mask = sum(1 << p for p in coalition)
    dt = torch.float64 if precise else torch.float32
    models = []
    for p_id in coalition:
        key = ocnn.shuffle_key(seed, mask, p_id)
        params = {k: v.to(dt).clone() for k, v in glob.items()}
        opt = KerasRMSprop(params, precise=precise)
        for t, rows in enumerate(ocnn.fedavg_round_rows(key, partner_rows[p_id], batch_sizes[p_id], M, e, m)):
            masks = step_masks(fedavg_drop_key(key, e, m, t), len(rows))
            g, _ = gradients(params, data.x_train[rows], data.y_train[rows], masks, dtype=dt if precise else None)
            opt.step(params, g)
        models.append(params)
    return models


def evaluate(p, x, y, batch=500):
    """[mean CE, accuracy] like Keras evaluate in inference mode."""
    torch = _torch()
    correct, loss = 0, 0.0
    with torch.no_grad():
        for s in range(0, len(y), batch):
            z = forward(p, x[s:s + batch])
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
            return torch.from_numpy(np.ascontiguousarray(x.reshape(x.shape[0], 32, 32, 3)))
        self.x_train, self.y_train = img(x_train), lab(y_train)
        self.x_val, self.y_val = img(x_val), lab(y_val)
        self.x_test, self.y_test = img(x_test), lab(y_test)


class _FitLog(ocnn._FitLog):
    """Keras fit history of one fit (see oracle/cnn.py _FitLog): the training forward runs with the step's
    dropout masks, as Keras' fit reports it; val metrics in inference mode."""

    def batch(self, params, x, y, loss_mean, masks=None):
        torch = _torch()
        with torch.no_grad():
            self.correct += int((forward(params, x, masks).argmax(1) == y).sum())
        self.loss += loss_mean * len(y)
        self.n += len(y)

    def store(self, h, e, m, params, data):
        vl, va = evaluate(params, data.x_val, data.y_val)
        h["val_loss"][e, m], h["val_accuracy"][e, m] = vl, va
        h["loss"][e, m] = self.loss / self.n if self.n else np.nan
        h["accuracy"][e, m] = self.correct / self.n if self.n else np.nan


def coalition_value(data, partner_rows, batch_sizes, coalition, seed=0, epochs=1, M=10,
                    aggregation="data-volume", early_stopping=False, return_model=False, approach="fedavg",
                    history=None):
    """v(S) of one coalition, the reference's way (sequential), on the engine's keyed init, order and masks.
    With a `history` dict, the learning history (mplc/mpl_utils.py:11-27) is recorded into it."""
    torch = _torch()
    coalition = tuple(sorted(coalition))
    mask = sum(1 << p for p in coalition)
    glob = unpack(init_params(ocnn.init_key(seed, mask)))
    epochs_done = epochs
    if history is not None:
        for p_id in coalition:
            history[p_id] = {k: np.full((epochs, M), np.nan) for k in ocnn.HISTORY_METRICS}
        if len(coalition) > 1:
            history["mpl_model"] = {"val_accuracy": np.zeros((epochs, M)), "val_loss": np.zeros((epochs, M))}
    log = None
    if len(coalition) == 1:
        p_id = coalition[0]
        key = ocnn.shuffle_key(seed, mask, p_id)
        params = {k: v.clone() for k, v in glob.items()}
        opt = KerasRMSprop(params)
        best, wait = np.inf, 0
        for e in range(epochs):
            log = _FitLog() if history is not None else None
            for t, rows in enumerate(ocnn.single_epoch_rows(key, partner_rows[p_id], batch_sizes[p_id], e)):
                masks = step_masks(single_drop_key(key, e, t), len(rows))
                g, lm = gradients(params, data.x_train[rows], data.y_train[rows], masks)
                if log is not None:
                    log.batch(params, data.x_train[rows], data.y_train[rows], lm, masks)
                opt.step(params, g)
            if early_stopping and epochs > PATIENCE:
                vl, _ = evaluate(params, data.x_val, data.y_val)
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
        w = [1 / len(coalition)] * len(coalition) if aggregation == "uniform" else np.asarray(sizes) / np.sum(sizes)
        val_hist = []
        for e in range(epochs):
            if early_stopping and epochs > PATIENCE:
                val_hist.append(evaluate(glob, data.x_val, data.y_val)[0])
            for m in range(M):
                if history is not None:  # round-start collective model (eval_and_log_model_val_perf)
                    vl, va = evaluate(glob, data.x_val, data.y_val)
                    history["mpl_model"]["val_loss"][e, m], history["mpl_model"]["val_accuracy"][e, m] = vl, va
                if approach != "fedavg":  # sequential approaches, as oracle/cnn.py
                    params = {k: v.clone() for k, v in glob.items()}
                    opt = KerasRMSprop(params)
                    snaps = [None] * len(coalition)
                    for mi in ocnn.seq_member_order(seed, mask, len(coalition), e, m):
                        p_id = coalition[mi]
                        key = ocnn.shuffle_key(seed, mask, p_id)
                        steps = ocnn.fedavg_round_rows(key, partner_rows[p_id], batch_sizes[p_id], M, e, m)
                        log = _FitLog() if history is not None else None
                        for t, rows in enumerate(steps):
                            masks = step_masks(fedavg_drop_key(key, e, m, t), len(rows))
                            g, lm = gradients(params, data.x_train[rows], data.y_train[rows], masks)
                            if log is not None:
                                log.batch(params, data.x_train[rows], data.y_train[rows], lm, masks)
                            opt.step(params, g)
                        snaps[mi] = {k: v.clone() for k, v in params.items()}
                        if log is not None:
                            log.store(history[p_id], e, m, params, data)
                    if approach == "seqavg" or (approach == "seq-with-final-agg" and m == M - 1):
                        glob = ocnn.average_models(glob, snaps, w)
                    else:
                        glob = params
                    continue
                partner_models = []
                for p_id in coalition:
                    key = ocnn.shuffle_key(seed, mask, p_id)
                    params = {k: v.clone() for k, v in glob.items()}
                    opt = KerasRMSprop(params)  # fresh optimizer per partner fit
                    steps = ocnn.fedavg_round_rows(key, partner_rows[p_id], batch_sizes[p_id], M, e, m)
                    log = _FitLog() if history is not None else None
                    for t, rows in enumerate(steps):
                        masks = step_masks(fedavg_drop_key(key, e, m, t), len(rows))
                        g, lm = gradients(params, data.x_train[rows], data.y_train[rows], masks)
                        if log is not None:
                            log.batch(params, data.x_train[rows], data.y_train[rows], lm, masks)
                        opt.step(params, g)
                    if log is not None:
                        log.store(history[p_id], e, m, params, data)
                    partner_models.append(params)
                new = {}
                for k in glob:
                    stack = np.array([pm[k].numpy() for pm in partner_models])
                    new[k] = torch.from_numpy(np.average(stack, axis=0, weights=w).astype(np.float32))
                glob = new
            if early_stopping and epochs > PATIENCE and e >= PATIENCE and val_hist[e] > val_hist[e - PATIENCE]:
                epochs_done = e + 1
                break
    _, acc = evaluate(glob, data.x_test, data.y_test)
    if return_model:
        return acc, epochs_done, pack(glob)
    return acc, epochs_done
