"""Host driver of the batched MNIST CNN trainer (csrc/mnist_cnn.hip, include/mplc_hip_cnn.h).

Trains a batch of coalitions at once and returns their test accuracies.  Semantics follow the
reference's learning path for the MNIST model (mplc/dataset.py:457-479):
  FedAvg coalition (|S| >= 2), mplc/multi_partner_learning.py:195-216, 285-334:
    init random model; per epoch, each partner's rows are permuted and split into M minibatches
    (mplc/partner.py:155-167); per round m every partner starts from the global model with a FRESH Adam
    and runs ceil(L_m / bs_p) steps of bs_p samples (Keras fit, 1 epoch, shuffled); the round ends with
    the data-volume (or uniform) weighted average (mplc/mpl_utils.py:90-115) -> next global model.
    Early stopping (when enabled and E > PATIENCE): val loss of the global model at the start of epoch e
    compared with epoch e - 10 (mplc/multi_partner_learning.py:177-193).
  Singleton (|S| == 1), mplc/multi_partner_learning.py:238-269: one Keras fit over all rows, E epochs,
    batch bs_p, persistent Adam, Keras EarlyStopping(val_loss, patience=10).
  v(S) = test accuracy of the final model (mplc/multi_partner_learning.py:158-169).
"""
import ctypes

import numpy as np

from . import _native
from .fedavg import aggregation_weights

STRIDE = 1199936
NPARAM = 1199882
FEAT = 9216
HID = 128
W1P = 320
W2P = 18496
W1_BANDS = 3  # MPLC_CNN_W1_BANDS: [dW1 | db1] partials per sample (data-gradient blocks)
W2T = 32768  # MPLC_CNN_W2T: W2 in Winograd form (forward), then transposed (data gradient)
WG_SAMPLES = 9  # samples per conv2 weight-gradient split; the library's value replaces it at bind time
ADAM_LAST = 1 << 30  # adam_t flag (csrc/mnist_cnn.hip): the optimizer's last step
PROF_ALL = -1        # mplc_cnn_train_t.prof_kernel (MPLC_PROF_ALL): time every launch of the step
PATIENCE = 10

# Keras get_weights() order of the MNIST model (mplc/dataset.py:460-471): (offset in a model row, shape)
KERAS_LAYERS = ((0, (3, 3, 1, 32)), (288, (32,)), (320, (3, 3, 32, 64)), (18752, (64,)), (18816, (9216, 128)),
                (1198464, (128,)), (1198592, (128, 10)), (1199872, (10,)))


def keras_weights(row, layers=KERAS_LAYERS):
    """A model row (fp32, this engine's layout) as the list of arrays Keras' get_weights() returns."""
    row = np.asarray(row, dtype=np.float32)
    return [row[off:off + int(np.prod(shape))].reshape(shape).copy() for off, shape in layers]


REP_IDLE, REP_FEDAVG, REP_SINGLE, REP_SEQ = -1, 0, 1, 2
SEQ_REC = 6
SEQ_APPROACHES = ("seq-pure", "seq-with-final-agg", "seqavg")
M64 = (1 << 64) - 1


class ReplicaT(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("n_rows", ctypes.c_int32), ("batch", ctypes.c_int32),
                ("rows_off", ctypes.c_int32), ("split_off", ctypes.c_int32), ("model", ctypes.c_int32),
                ("key", ctypes.c_uint64)]


assert ctypes.sizeof(ReplicaT) == 32

REPLICA_DTYPE = np.dtype([("kind", np.int32), ("n_rows", np.int32), ("batch", np.int32), ("rows_off", np.int32),
                          ("split_off", np.int32), ("model", np.int32), ("key", np.uint64)])
assert REPLICA_DTYPE.itemsize == 32


class TrainT(ctypes.Structure):
    _fields_ = [("n_rep", ctypes.c_int32), ("bmax", ctypes.c_int32), ("w2_splits", ctypes.c_int32),
                ("pad0", ctypes.c_int32), ("step", ctypes.c_int32), ("minibatch_count", ctypes.c_int32),
                ("round_len", ctypes.c_int32), ("epochs", ctypes.c_int32),
                ("reps", ctypes.c_void_p), ("rows", ctypes.c_void_p), ("splits", ctypes.c_void_p),
                ("seq", ctypes.c_void_p),
                ("x", ctypes.c_void_p), ("labels", ctypes.c_void_p),
                ("params", ctypes.c_void_p), ("adam_m", ctypes.c_void_p), ("adam_v", ctypes.c_void_p),
                ("idx", ctypes.c_void_p), ("cnt", ctypes.c_void_p), ("adam_t", ctypes.c_void_p),
                ("pooled", ctypes.c_void_p), ("code", ctypes.c_void_p), ("hidden", ctypes.c_void_p),
                ("dhidden", ctypes.c_void_p), ("dpooled", ctypes.c_void_p), ("w1_part", ctypes.c_void_p),
                ("w2_part", ctypes.c_void_p), ("w2t", ctypes.c_void_p),
                ("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("eps", ctypes.c_float), ("prof_kernel", ctypes.c_int32), ("phases", ctypes.c_int32),
                ("prof_begin", ctypes.c_void_p), ("prof_end", ctypes.c_void_p), ("hstats", ctypes.c_void_p),
                ("glob", ctypes.c_void_p), ("rep_glob", ctypes.c_void_p), ("w3src", ctypes.c_void_p),
                ("avg_n", ctypes.c_int32), ("pad1", ctypes.c_int32), ("avg_first", ctypes.c_void_p),
                ("avg_w", ctypes.c_void_p), ("avg_scale", ctypes.c_void_p), ("avg_glob", ctypes.c_void_p),
                ("avg_out", ctypes.c_void_p), ("avg_rep", ctypes.c_void_p)]

KERNEL_IDS = {"conv_fwd": 1, "dense_fwd": 2, "head": 3, "dense1_bwd_adam": 4, "conv_bwd_data": 5, "conv_wgrad": 6,
              "adam_small": 7}


_BOUND = False


def _bind():
    global _BOUND
    if _BOUND:
        return
    c_int, c_int64, vp = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p
    _native.register("mplc_cnn_stride", c_int, [])
    _native.register("mplc_cnn_init_params", c_int, [vp, c_int64, vp, c_int, vp])
    _native.register("mplc_cnn_copy_rows", c_int, [vp, vp, c_int64, vp, c_int, vp])
    _native.register("mplc_cnn_train_step", c_int, [ctypes.POINTER(TrainT), vp])
    _native.register("mplc_cnn_evaluate", c_int, [vp, c_int64, c_int, vp, vp, c_int, c_int, vp, vp, vp, vp, vp, vp])
    lib = _native.lib()
    global WG_SAMPLES
    WG_SAMPLES = int(lib.mplc_cnn_wgrad_split_samples())  # the library's conv2 weight-gradient split size
    _native.check_layout(lib.mplc_cnn_layout, layout_items(), "MNIST CNN")
    _BOUND = True


def layout_items():
    """The host's view of every MPLC_CNN_Q_* layout item (include/mplc_hip_cnn.h): name -> (query id, value)."""
    return {"STRIDE": (0, STRIDE), "NPARAM": (1, NPARAM), "FEAT": (2, FEAT), "HID": (3, HID), "W1P": (4, W1P),
            "W2P": (5, W2P), "W2T": (6, W2T), "W1_BANDS": (7, W1_BANDS), "WG_SAMPLES": (8, WG_SAMPLES),
            "PROF_KERNELS": (9, len(KERNEL_IDS)), "TRAIN_T_BYTES": (10, ctypes.sizeof(TrainT)),
            "REPLICA_T_BYTES": (11, ctypes.sizeof(ReplicaT))}


# ------------------------------------------------------------------------------------------------
# keys (restated bit for bit in oracle/cnn.py)
# ------------------------------------------------------------------------------------------------
def mix64(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
    return z ^ (z >> 31)


def init_key(seed, mask):
    return mix64(mix64((seed + 0x1517) & M64) ^ mask)


def shuffle_key(seed, mask, partner):
    return mix64(mix64(mix64((seed + 0x5EED) & M64) ^ mask) ^ (partner + 1))


def seq_order_key(seed, mask):
    """Key of the per-round member order of a sequential coalition (keyed.h seq_locate)."""
    return mix64(mix64((seed + 0x5E90) & M64) ^ mask)


def subkey(key, a, b):
    return mix64(key ^ mix64(((a << 32) | b) & M64))


def keyed_perm(key, n, i):
    """Host restatement of keyed.h keyed_perm: bijection of [0, n) (4-round Feistel + cycle walking)."""
    if n <= 1:
        return 0
    h = ((n - 1).bit_length() + 1) >> 1
    mask = (1 << h) - 1
    x = i
    while True:
        L, R = x >> h, x & mask
        for rd in range(4):
            L, R = R, L ^ (mix64(key ^ (rd << 40) ^ R) & mask)
        x = (L << h) | R
        if x < n:
            return x


def seq_member_order(seed, mask, k, e, m):
    """Member indices (ascending-partner order) of a sequential coalition in the visiting order of round
    (e, m) (keyed.h seq_locate)."""
    okey = subkey(seq_order_key(seed, mask), 0x60000 + e, m)
    return [keyed_perm(okey, k, idx) for idx in range(k)]


def _i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


def torch_i32(values, device):
    import torch
    return torch.tensor(list(values), dtype=torch.int32, device=device)


def minibatch_bounds(n, M):
    """[0, int(1/M*n), ..., int((M-1)/M*n), n] exactly as np.split's indices in mplc/partner.py:159-167."""
    split_indices = np.arange(1, M + 1) / M
    inner = (split_indices[:-1] * n).astype(int)
    return [0] + [int(v) for v in inner] + [int(n)]


EVAL_BLOCK = 256  # the evaluation kernels sum the loss in fixed blocks of this many samples


def eval_plan(n, C, sample_bytes, model_bytes, budget):
    """(chunk, group) of an evaluation of C models on n samples within `budget` bytes of workspace: models are
    evaluated `group` at a time, each chunk of samples holding sample_bytes per (model, sample) plus model_bytes
    per model.  Every chunk but the last is a multiple of EVAL_BLOCK samples, so the kernels' loss sums (fixed
    256-sample blocks in sample order, mplc_cnn_evaluate / mplc_cifar_evaluate) do not depend on C, the budget or
    which models share the evaluation: a model's val loss - what the early-stopping rule compares - is a function
    of the model alone."""
    cap = max(0, budget - C * model_bytes) // max(1, C * sample_bytes)
    if cap >= n and n <= 65535:
        return n, C
    if cap >= EVAL_BLOCK:
        return min(cap, 65535) // EVAL_BLOCK * EVAL_BLOCK, C
    chunk = min(n, EVAL_BLOCK)
    group = max(1, budget // (chunk * sample_bytes + model_bytes))
    return chunk, min(C, group)


class MnistModel:
    """Model hooks of the batched MNIST CNN (csrc/mnist_cnn.hip): parameter layout, optimizer state,
    workspaces, one lockstep step, evaluation.  TrainBatch / CnnBatchTrainer drive any model with these."""
    name = "mnist_cnn"
    STRIDE, NPARAM = STRIDE, NPARAM
    EVAL_SAMPLE_BYTES, EVAL_MODEL_BYTES = (FEAT + HID) * 4, W2T * 4  # evaluation workspace (mplc_cnn_evaluate)
    KERAS_LAYERS = KERAS_LAYERS
    KERNEL_IDS = KERNEL_IDS
    input_shape = (28, 28)
    # FedAvg aggregation leaves W3 (98 % of the parameters) out of the broadcast: a round's first step reads
    # it from the coalition row (mplc_cnn_train_t.glob, mplc_fedavg_aggregate_bcast_skip)
    BCAST_SKIP = (KERAS_LAYERS[4][0], KERAS_LAYERS[5][0])
    # ... and the round's last step can average it in its dense pass (mplc_cnn_train_t.avg_*, ABI 4): the
    # aggregation then skips that range altogether (mplc_fedavg_aggregate_skip)
    FUSE_AVG = True

    def __init__(self):
        _bind()
        self.lib = _native.lib()

    def replica_bytes(self, bmax):
        return (3 * STRIDE * 4 + bmax * FEAT * 9 + 2 * bmax * HID * 4 + W1_BANDS * bmax * W1P * 4 + ((bmax + WG_SAMPLES - 1) // WG_SAMPLES) * W2P * 4
                + W2T * 4 + bmax * 12)

    def init_params(self, glob, keys, stream):
        _native.check(self.lib.mplc_cnn_init_params(_native.ptr(glob), STRIDE, _native.ptr(keys), glob.shape[0], stream),
                      "mplc_cnn_init_params")

    def alloc(self, st):
        """Optimizer state, workspaces and the step struct of a TrainBatch (params already set)."""
        import torch
        eng, dev, R, B = st.eng, st.dev, st.R, st.bmax
        f32 = dict(dtype=torch.float32, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        opt = getattr(st, "resume_opt", None)  # a compacted batch continues its replicas' moments
        st.adam_m = opt["adam_m"] if opt else torch.zeros((R, STRIDE), **f32)
        st.adam_v = opt["adam_v"] if opt else torch.zeros((R, STRIDE), **f32)
        splits = (B + WG_SAMPLES - 1) // WG_SAMPLES
        st.ws = dict(
            idx=torch.empty((R, B), **i32), cnt=torch.empty(R, **i32), adam_t=torch.empty(R, **i32),
            pooled=torch.empty((R, B, FEAT), **f32), code=torch.empty((R, B, FEAT), dtype=torch.uint8, device=dev),
            hidden=torch.empty((R, B, HID), **f32), dhidden=torch.empty((R, B, HID), **f32),
            dpooled=torch.empty((R, B, FEAT), **f32), w1_part=torch.empty((R, B, W1_BANDS, W1P), **f32),
            w2_part=torch.empty((R, splits, W2P), **f32), w2t=torch.empty((R, W2T), **f32),
            w3src=torch.empty(R, **i32))
        t = TrainT()
        t.n_rep, t.bmax, t.w2_splits = R, B, splits
        t.minibatch_count, t.round_len, t.epochs = eng.minibatch_count, st.round_len, st.epochs
        t.reps, t.rows, t.splits = st.rep_t.data_ptr(), eng.rows_d.data_ptr(), eng.splits_d.data_ptr()
        t.seq = st.seq_t.data_ptr() if st.seq_t is not None else None
        t.x, t.labels = eng.x_train_d.data_ptr(), eng.y_train_d.data_ptr()
        t.params, t.adam_m, t.adam_v = st.params.data_ptr(), st.adam_m.data_ptr(), st.adam_v.data_ptr()
        for k, v in st.ws.items():
            setattr(t, k, v.data_ptr())
        t.lr, t.beta1, t.beta2, t.eps = 0.001, 0.9, 0.999, 1e-7
        if not st.seq_mode:  # FedAvg rounds start from the coalition row (W3 is not broadcast)
            t.glob, t.rep_glob = st.glob.data_ptr(), st.src_map.data_ptr()
        st.t = t

    def free(self, st):
        st.adam_m = st.adam_v = None

    @staticmethod
    def opt_state(st):
        """The per-replica optimizer rows of a TrainBatch (Adam moments)."""
        return {"adam_m": st.adam_m, "adam_v": st.adam_v}

    def step(self, st, s, prof):
        st.t.step = s
        if prof is not None:
            if prof.all:
                prof.bind(self.KERNEL_IDS)
            ev0, ev1 = prof.pair()
            st.t.prof_kernel = PROF_ALL if prof.all else self.KERNEL_IDS[prof.kernel]
            st.t.prof_begin, st.t.prof_end = ev0, ev1
        else:
            st.t.prof_kernel, st.t.prof_begin, st.t.prof_end = 0, None, None
        fused = st.fused_step(s)  # the round's last step: W3's average in the dense pass
        st.t.avg_n = st.avg["n"] if fused else 0
        _native.check(self.lib.mplc_cnn_train_step(ctypes.byref(st.t), st.stream), "mplc_cnn_train_step")
        if prof is not None and prof.want_stash:
            prof.stash_step(st.ws["cnt"], st.ws["adam_t"], st.ws["w3src"],
                            st.avg["rep"] if fused else st.avg_none)

    @staticmethod
    def algorithmic_units(stash):
        """Algorithmic work of the timed steps from their stashed schedules [(cnt, adam_t, w3src)], per kernel:
        samples (the convolution kernels' unit) and the HBM bytes the two W3 kernels must move
        (csrc/mnist_cnn.hip dense_fwd_kernel / dense1_bwd_adam_kernel):
          dense_fwd:       W3 read + per sample its pooled row read and hidden row written;
          dense1_bwd_adam: W3 read and written; Adam moments by the optimizer step t - t = 1 writes the
                           gradient into the m slot, t = 2 reads it and writes m and v, t >= 3 reads and
                           writes m and v, the optimizer's last step writes no moments; per sample the pooled
                           row and dh read, the dpooled row written.
        A FedAvg round's first step reads W3 from the coalition row (w3src >= 0), shared by the coalition's
        replicas: that row counts once per coalition, not once per replica."""
        import torch
        if not stash:
            return {}
        # one step at a time: the replica count differs between lockstep batches when the memory budget splits
        # a job into several (the per-step copies then have different lengths)
        w3 = float(FEAT * HID * 4)
        samples = d1_bytes = df_bytes = 0.0
        for rec in stash:
            cnt, at, src = rec[:3]
            fused = rec[3] if len(rec) > 3 else torch.zeros_like(cnt)  # 1 + fused coalition index, or 0
            cnt = cnt.to(torch.float64)
            shared = src >= 0
            # distinct coalition rows read by this step's first-step replicas
            n_shared_rows = float(torch.unique(src[shared & (cnt > 0)]).numel())
            t = at & (ADAM_LAST - 1)
            last = (at & ADAM_LAST) != 0
            act = (cnt > 0).to(torch.float64)
            mom_rd = torch.where(t == 1, 0.0, torch.where(t == 2, 1.0, 2.0)).to(torch.float64)
            mom_wr = torch.where(last, 0.0, torch.where(t == 1, 1.0, 2.0)).to(torch.float64)
            own = (~shared).to(torch.float64)  # replicas reading W3 from their own row
            # the W3 store: the replica's own row, or for a fused coalition (the round's last step) one coalition
            # row per coalition, and its members idle this step read their final rows into the average
            wr = (fused == 0).to(torch.float64)
            idle_fused = float(((fused > 0) & (cnt == 0)).sum().item())
            n_avg_rows = float(torch.unique(fused[fused > 0]).numel())
            d1 = act * (w3 * (wr + own + mom_rd + mom_wr) + cnt * float(2 * FEAT * 4 + HID * 4))
            df = act * (w3 * own + cnt * float(FEAT * 4 + HID * 4))
            samples += float(cnt.sum().item())
            d1_bytes += float(d1.sum().item()) + (n_shared_rows + n_avg_rows + idle_fused) * w3
            df_bytes += float(df.sum().item()) + n_shared_rows * w3
        return {"samples": samples, "dense1_bwd_adam_bytes": d1_bytes, "dense_fwd_bytes": df_bytes}

    def evaluate(self, eng, sel, x, y):
        """(correct counts, mean CE) of the C models in `sel` [C][STRIDE] on (x, y)."""
        import torch
        dev = eng.device
        stream = _native.stream_handle(dev)
        n = int(y.numel())
        C = sel.shape[0]
        chunk, group = eval_plan(n, C, self.EVAL_SAMPLE_BYTES, self.EVAL_MODEL_BYTES, eng.eval_budget_bytes)
        pooled = torch.empty((group, chunk, FEAT), dtype=torch.float32, device=dev)
        hidden = torch.empty((group, chunk, HID), dtype=torch.float32, device=dev)
        correct = torch.zeros(C, dtype=torch.int32, device=dev)
        loss = torch.zeros(C, dtype=torch.float64, device=dev)
        wino = torch.empty((group, W2T), dtype=torch.float32, device=dev)
        for g0 in range(0, C, group):
            g = min(group, C - g0)
            _native.check(self.lib.mplc_cnn_evaluate(_native.ptr(sel[g0:g0 + g]), STRIDE, g, _native.ptr(x),
                                                     _native.ptr(y), n, chunk, _native.ptr(pooled), _native.ptr(hidden),
                                                     _native.ptr(wino), _native.ptr(correct[g0:g0 + g]),
                                                     _native.ptr(loss[g0:g0 + g]), stream), "mplc_cnn_evaluate")
        return correct.cpu().numpy().astype(np.float64), loss.cpu().numpy() / n


def schedule_geometry(eng, coalitions, epochs, seq_mode=False):
    """(round_len, fed_steps, total_steps) of a lockstep batch: the longest partner fit of any round (FedAvg; the
    members' fits back to back for the sequential approaches), the FedAvg steps and the steps the batch runs."""
    sizes, M = eng.partner_sizes, eng.minibatch_count
    round_len, single_steps = 1, 0
    for coal in coalitions:
        if len(coal) == 1:
            p = coal[0]
            single_steps = max(single_steps, epochs * -(-sizes[p] // eng.batch_sizes[p]))
        elif seq_mode:  # the members' fits run back to back inside a round
            for m in range(M):
                round_len = max(round_len, sum(-(-(eng.bounds[p][m + 1] - eng.bounds[p][m]) // eng.batch_sizes[p])
                                               for p in coal))
        else:
            for p in coal:
                b = eng.bounds[p]
                for m in range(M):
                    round_len = max(round_len, -(-(b[m + 1] - b[m]) // eng.batch_sizes[p]))
    fed_steps = epochs * M * round_len if any(len(c) > 1 for c in coalitions) else 0
    return round_len, fed_steps, max(fed_steps, single_steps)


class TrainBatch:
    """Device state of one lockstep batch: coalition global rows, replica rows, optimizer state, workspaces
    (model-specific parts through eng.model_impl)."""

    def __init__(self, eng, coalitions, epochs, lib, record=False, resume=None):
        """resume (CnnBatchTrainer._compact): continue coalitions of an earlier batch - their coalition rows
        ("glob"), replica rows ("params") and optimizer rows ("opt", the model's opt_state names) in this batch's
        order, and that batch's schedule geometry ("round_len", "fed_steps", "total_steps": the step -> (epoch,
        round, position) map must not change, mplc_hip_cnn.h schedule)."""
        import torch
        self.eng, self.lib = eng, lib
        self.record = record
        self.model = eng.model_impl
        self.coalitions = coalitions
        self.epochs = epochs
        dev = eng.device
        self.dev = dev
        self.stream = _native.stream_handle(dev)
        C = len(coalitions)
        sizes = eng.partner_sizes
        self.approach = getattr(eng, "approach", "fedavg")
        seq_mode = self.approach in SEQ_APPROACHES
        reps, src, first, single, seq_recs, snap_first = [], [], [], [], [], []
        for ci, coal in enumerate(coalitions):
            mask = sum(1 << p for p in coal)
            first.append(len(reps))
            single.append(len(coal) == 1)
            if seq_mode and len(coal) > 1:
                # one model per coalition; member records in ascending partner order (the partners_list order)
                off = len(seq_recs)
                for p in coal:
                    key = shuffle_key(eng.seed, mask, p)
                    seq_recs.extend([sizes[p], eng.batch_sizes[p], eng.rows_off[p], eng.split_off[p],
                                     _i32(key & 0xFFFFFFFF), _i32(key >> 32)])
                snap_first.append(sum(len(coalitions[c]) for c in range(ci) if len(coalitions[c]) > 1))
                reps.append((REP_SEQ, len(coal), max(eng.batch_sizes[p] for p in coal), off, 0, len(reps),
                             seq_order_key(eng.seed, mask)))
                src.append(ci)
                continue
            for p in coal:
                reps.append((REP_SINGLE if len(coal) == 1 else REP_FEDAVG, sizes[p], eng.batch_sizes[p],
                             eng.rows_off[p], eng.split_off[p], len(reps), shuffle_key(eng.seed, mask, p)))
                src.append(ci)
                snap_first.append(0)
        first.append(len(reps))
        self.coal_first, self.coal_is_single = first, single
        self.seq_mode = seq_mode
        R = len(reps)
        self.R, self.C = R, C
        self.rep_arr = np.zeros(R, dtype=REPLICA_DTYPE)
        for i, rp in enumerate(reps):
            self.rep_arr[i] = rp
        self.bmax = int(max(eng.batch_sizes[p] for coal in coalitions for p in coal))
        self.round_len, self.fed_steps, self.total_steps = schedule_geometry(eng, coalitions, epochs, seq_mode)
        if resume is not None:
            self.round_len, self.fed_steps, self.total_steps = (resume["round_len"], resume["fed_steps"],
                                                                resume["total_steps"])
        S = self.model.STRIDE
        f32 = dict(dtype=torch.float32, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.f32, self.i32 = f32, i32
        src_map = torch.tensor(src, **i32)
        self.src_map = src_map  # replica -> coalition row of glob
        if resume is not None:
            self.glob, self.params = resume["glob"], resume["params"]
            assert tuple(self.glob.shape) == (C, S) and tuple(self.params.shape) == (R, S)
        else:
            self.glob = torch.empty((C, S), **f32)
            self.params = torch.empty((R, S), **f32)
            keys = torch.from_numpy(np.array([init_key(eng.seed, sum(1 << p for p in c)) for c in coalitions],
                                             dtype=np.uint64).view(np.int64)).to(dev)
            self.model.init_params(self.glob, keys, self.stream)
            _native.check(lib.mplc_cnn_copy_rows(_native.ptr(self.params), _native.ptr(self.glob), S,
                                                 _native.ptr(src_map), R, self.stream), "mplc_cnn_copy_rows")
        self.rep_t = torch.from_numpy(self.rep_arr.view(np.uint8).copy()).to(dev)
        self.seq_t = torch.tensor(seq_recs, **i32) if seq_recs else None
        self.snap = None
        if seq_mode and (self.approach != "seq-pure" or record) and seq_recs:
            # partner.model_weights of the aggregating variants: one snapshot row per (coalition, member)
            self.snap = torch.zeros((len(seq_recs) // SEQ_REC, S), **f32)
            self.snap_first_t = torch.tensor(snap_first, **i32)
        self.resume_opt = resume["opt"] if resume is not None else None  # alloc() takes these rows over
        self.model.alloc(self)
        self.resume_opt = None
        self.hstats = None
        if record:  # per-step training loss / accuracy sums of every replica (the head kernel's hstats)
            self.hstats = torch.zeros((R, 3), dtype=torch.float64, device=dev)
            self.t.hstats = self.hstats.data_ptr()
        self.stopped = np.zeros(C, dtype=bool)
        self.kind_host = self.rep_arr["kind"].copy()
        self.avg = {"n": 0}
        self.avg_none = torch.zeros(R, **i32)  # the stash's "no fused coalition" record (bench accounting)
        self.run_args = self.make_runs()

    def make_runs(self):
        """FedAvg aggregation launches: one per contiguous run of live FedAvg coalitions (a coalition's replica
        rows are contiguous; singletons and stopped coalitions break runs)."""
        import torch
        runs, cur = [], []
        for ci in range(self.C):
            if self.coal_is_single[ci] or self.stopped[ci]:
                if cur:
                    runs.append(cur)
                cur = []
            else:
                cur.append(ci)
        if cur:
            runs.append(cur)
        sizes = self.eng.partner_sizes
        # aggregation inputs: FedAvg replica rows, or the SEQ snapshot rows (members contiguous per coalition)
        if self.seq_mode:
            first, acc = [], 0
            for ci in range(self.C):
                first.append(acc)
                acc += len(self.coalitions[ci]) if not self.coal_is_single[ci] else 0
            first.append(acc)
        else:
            first = self.coal_first
        # every run's offsets, weights and scales go to the device in one copy per dtype (views per run): an early-
        # stopping epoch end rebuilds the runs, and per-run copies stalled the stream for tens of microseconds each
        f_all, f64_all, spans = [], [], []
        for run in runs:
            f = [first[ci] - first[run[0]] for ci in run] + [first[run[-1] + 1] - first[run[0]]]
            w, sc = [], []
            for ci in run:
                ww, scl = aggregation_weights([sizes[p] for p in self.coalitions[ci]], self.eng.aggregation)
                w.extend(ww)
                sc.append(scl)
            spans.append((len(f_all), len(f), len(f64_all), len(w), len(sc)))
            f_all.extend(f)
            f64_all.extend(w)
            f64_all.extend(sc)
        f_dev = torch.tensor(f_all, **self.i32) if f_all else None
        x_dev = torch.tensor(f64_all, dtype=torch.float64, device=self.dev) if f64_all else None
        args = []
        for run, (fo, fn, xo, wn, sn) in zip(runs, spans):
            # the broadcast may skip W3 / W5 only if every member trains in every round: a round's first step
            # is what reloads them from the coalition row, and a partner with an empty minibatch (fewer rows
            # than minibatch_count) has no step in that round, yet enters the average with the round's global
            # model (the reference's fresh model from the global weights, mplc/multi_partner_learning.py:319)
            full_bcast = any(self.eng.bounds[p][m + 1] == self.eng.bounds[p][m]
                             for ci in run for p in self.coalitions[ci] for m in range(self.eng.minibatch_count))
            args.append((self.coal_first[run[0]], run[0], len(run), f_dev[fo:fo + fn], x_dev[xo:xo + wn],
                         x_dev[xo + wn:xo + wn + sn], full_bcast))
        return self._fuse_runs(args)

    def _fuse_runs(self, args):
        """Runs whose W3 average the round's last step computes in its dense pass (mplc_cnn_train_t.avg_*, ABI 4):
        FedAvg runs that broadcast with W3 skipped, for a model with the fused kernel, without history recording
        (the partners' val evaluations read the replicas' own W3 rows, which a fused step does not write).  Each
        run's tuple gains a flag; the step's tables cover all fused runs of the batch."""
        import torch
        eng = self.eng
        ok = (getattr(self.model, "FUSE_AVG", False) and not self.seq_mode and eng.bcast_skip and not self.record
              and getattr(eng, "fuse_avg", True))
        out, first, rep_w, scale, glob_row = [], [], np.zeros(self.R), [], []
        rep = np.zeros(self.R, dtype=np.int32)
        sizes = eng.partner_sizes
        for (r0, c0, nc, f, w, sc, full_bcast) in args:
            fuse = bool(ok and not full_bcast)
            out.append((r0, c0, nc, f, w, sc, full_bcast, fuse))
            if not fuse:
                continue
            for ci in range(c0, c0 + nc):
                b, e = self.coal_first[ci], self.coal_first[ci + 1]
                ww, scl = aggregation_weights([sizes[p] for p in self.coalitions[ci]], eng.aggregation)
                rep_w[b:e] = ww
                rep[b:e] = len(scale) + 1
                first.extend([b, e])
                scale.append(scl)
                glob_row.append(ci)
        if not scale:
            self.avg = {"n": 0}
            return out
        dev = self.dev
        self.avg = {"n": len(scale), "first": torch.tensor(first, **self.i32),
                    "w": torch.from_numpy(rep_w).to(dev), "scale": torch.tensor(scale, dtype=torch.float64, device=dev),
                    "glob": torch.tensor(glob_row, **self.i32), "rep": torch.from_numpy(rep).to(dev)}
        t = self.t
        t.avg_first, t.avg_w, t.avg_scale = (self.avg["first"].data_ptr(), self.avg["w"].data_ptr(),
                                             self.avg["scale"].data_ptr())
        t.avg_glob, t.avg_out, t.avg_rep = (self.avg["glob"].data_ptr(), self.glob.data_ptr(),
                                            self.avg["rep"].data_ptr())
        return out

    def fused_step(self, s):
        """Step s is the last step of a FedAvg round and the batch has fused runs: the step averages their W3."""
        return (self.avg["n"] > 0 and self.fed_steps > 0 and s < self.fed_steps
                and (s + 1) % self.round_len == 0)

    def step(self, s):
        self.model.step(self, s, self.eng.profiler)
        if self.snap is not None:
            t = self.t
            _native.check(self.lib.mplc_seq_snapshot(_native.ptr(self.params), self.model.STRIDE, self.model.NPARAM,
                                                     _native.ptr(self.rep_t), self.R, _native.ptr(self.seq_t),
                                                     ctypes.c_void_p(t.splits), s, t.minibatch_count, t.round_len,
                                                     t.epochs, _native.ptr(self.snap_first_t), _native.ptr(self.snap),
                                                     self.stream), "mplc_seq_snapshot")

    def _rows_copy(self, dst, src, mapping):
        m = torch_i32(mapping, self.dev)
        _native.check(self.lib.mplc_cnn_copy_rows(_native.ptr(dst), _native.ptr(src), self.model.STRIDE, _native.ptr(m),
                                                  len(mapping), self.stream), "mplc_cnn_copy_rows")

    def aggregate(self, epoch_end=False):
        """End of a round.  fedavg: data-volume/uniform average of the partner models -> global, broadcast to
        the replicas (mplc/multi_partner_learning.py:300-311).  seq-pure: the model after the last member is
        the global model.  seqavg (every round) / seq-with-final-agg (epoch end): average of the members'
        snapshots -> global -> the coalition model (mplc/multi_partner_learning.py:392-433)."""
        S, NP = self.model.STRIDE, self.model.NPARAM
        aggregate_now = (not self.seq_mode or self.approach == "seqavg"
                         or (self.approach == "seq-with-final-agg" and epoch_end))
        for (r0, c0, nc, first, w, sc, full_bcast, fused) in self.run_args:
            if aggregate_now:
                x = self.params[r0:] if not self.seq_mode else self.snap[self.snap_row(c0):]
                skip = None if (self.seq_mode or full_bcast or not self.eng.bcast_skip) else \
                    getattr(self.model, "BCAST_SKIP", None)
                if fused:  # the round's last step wrote W3's average into glob: the other layers only
                    _native.check(self.lib.mplc_fedavg_aggregate_skip(
                        _native.ptr(x), S, _native.ptr(first), _native.ptr(w), _native.ptr(sc), nc, NP,
                        _native.ptr(self.glob[c0:c0 + nc]), S, skip[0], skip[1], self.stream),
                        "mplc_fedavg_aggregate_skip")
                elif skip is not None:  # the next round's first step reads this range from glob
                    _native.check(self.lib.mplc_fedavg_aggregate_bcast_skip(
                        _native.ptr(x), S, _native.ptr(first), _native.ptr(w), _native.ptr(sc), nc, NP,
                        _native.ptr(self.glob[c0:c0 + nc]), S, skip[0], skip[1], self.stream),
                        "mplc_fedavg_aggregate_bcast_skip")
                else:
                    _native.check(self.lib.mplc_fedavg_aggregate(_native.ptr(x), S, _native.ptr(first), _native.ptr(w),
                                                                 _native.ptr(sc), nc, NP,
                                                                 _native.ptr(self.glob[c0:c0 + nc]), S,
                                                                 0 if self.seq_mode else 1, self.stream),
                                  "mplc_fedavg_aggregate")
                if self.seq_mode:  # the averaged model continues training
                    self._rows_copy(self.params[r0:r0 + nc], self.glob, list(range(c0, c0 + nc)))
            else:  # sequential without averaging: the coalition model as it stands
                self._rows_copy(self.glob[c0:c0 + nc], self.params, list(range(r0, r0 + nc)))

    def snap_row(self, ci):
        return sum(len(self.coalitions[c]) for c in range(ci) if not self.coal_is_single[c])

    def stop(self, cis):
        """Coalitions `cis` stop training (early stopping): their replicas go idle and the aggregation runs are
        rebuilt once for all of them (one epoch end can stop hundreds of coalitions)."""
        import torch
        for ci in cis:
            self.stopped[ci] = True
            self.kind_host[self.coal_first[ci]:self.coal_first[ci + 1]] = REP_IDLE
        ra = self.rep_arr.copy()
        ra["kind"] = self.kind_host
        self.rep_t.copy_(torch.from_numpy(ra.view(np.uint8).copy()).to(self.dev))
        self.run_args = self.make_runs()

    def release(self):
        """Drop every device buffer of this batch (compaction: the live rows were gathered first)."""
        self.params = self.glob = None
        self.model.free(self)
        self.ws = None
        self.t = None

    def finalize(self):
        """Singleton final models -> their coalition rows; free training state."""
        import torch
        S = self.model.STRIDE
        single = [ci for ci in range(self.C) if self.coal_is_single[ci]]
        if single:
            m = torch.tensor([self.coal_first[ci] for ci in single], **self.i32)
            tmp = torch.empty((len(single), S), **self.f32)
            _native.check(self.lib.mplc_cnn_copy_rows(_native.ptr(tmp), _native.ptr(self.params), S,
                                                      _native.ptr(m), len(single), self.stream), "mplc_cnn_copy_rows")
            self.glob[torch.tensor(single, device=self.dev)] = tmp
        self.params = None
        self.model.free(self)
        self.ws = None
        return self.glob


class CnnBatchTrainer:
    """Trains one batch of coalitions (all on the current HIP device) and evaluates them."""

    def __init__(self, engine):
        self.eng = engine
        self.lib = _native.lib()

    def prepare(self, coalitions, epochs, record=False):
        return TrainBatch(self.eng, coalitions, epochs, self.lib, record=record)

    # early stopping: once the replicas still training are at most this share of a lockstep batch, the batch is
    # compacted (CnnBatchTrainer._compact); 0 keeps every batch whole
    COMPACT_LIVE_SHARE = 0.75

    def run(self, coalitions, epochs, early_stopping, history=None, keep_models=False, started=False):
        """Train the coalitions in lockstep; returns (test accuracies, epochs done).  With `history` (a
        dict, one coalition only) the learning history is recorded into it (HistoryRecorder).  started: the
        batch's start was already reported to eng.progress (run_concurrent falling back to one stream).

        Early stopping leaves stopped coalitions' replicas idle in the lockstep batch; when the live replicas
        drop to COMPACT_LIVE_SHARE of the batch (FedAvg, several coalitions) the stopped coalitions' final models
        are test-evaluated and the live ones continue in a smaller batch (_compact): same rows, optimizer state
        and step schedule, so every v(S) is bit-identical to training without compaction."""
        eng = self.eng
        st = self.prepare(coalitions, epochs, record=history is not None)
        C = st.C
        rec = None
        if history is not None:
            if C != 1:
                raise ValueError("history recording takes exactly one coalition")
            rec = HistoryRecorder(self, st, epochs, history)
        sizes = eng.partner_sizes
        use_es = early_stopping and epochs > PATIENCE
        share = float(getattr(eng, "compact_live_share", self.COMPACT_LIVE_SHARE))
        compact = use_es and share > 0 and rec is None and not keep_models and not st.seq_mode
        orig = list(range(C))  # this batch's coalition index -> the caller's
        correct = np.zeros(C)
        # per coalition (the caller's index): epochs done, the val losses the stopping rule compared, Keras
        # EarlyStopping's best / wait
        epochs_done = np.full(C, epochs, dtype=np.int64)
        val_hist = [[] for _ in range(C)]
        es_best = np.full(C, np.inf)
        es_wait = np.zeros(C, dtype=np.int64)

        def layout(st):
            fed = [ci for ci in range(st.C) if not st.coal_is_single[ci]]
            spe = {ci: -(-sizes[st.coalitions[ci][0]] // eng.batch_sizes[st.coalitions[ci][0]])
                   for ci in range(st.C) if st.coal_is_single[ci]}
            return fed, spe
        fed, spe = layout(st)
        per_epoch_fed = eng.minibatch_count * st.round_len
        progress = getattr(eng, "progress", None)
        stats = eng.stats
        for s in range(st.total_steps):
            # replica-steps launched, and those of replicas still training (early stopping leaves the stopped
            # coalitions' replicas idle in the lockstep batch until it ends or is compacted)
            live_reps = int(np.sum(st.kind_host != REP_IDLE))
            if compact and 0 < live_reps < st.R and live_reps <= share * st.R:
                done = [ci for ci in range(st.C) if st.stopped[ci]]
                live = [ci for ci in range(st.C) if not st.stopped[ci]]
                correct[[orig[ci] for ci in done]] = self._final_correct(st, done)
                st = self._compact(st, live)
                orig = [orig[ci] for ci in live]
                fed, spe = layout(st)
                stats["compactions"] = stats.get("compactions", 0) + 1
            stats["replica_steps"] = stats.get("replica_steps", 0) + st.R
            stats["replica_steps_live"] = stats.get("replica_steps_live", 0) + live_reps
            if progress is not None and s % 30 == 0 and not (started and s == 0):
                progress(s, st.total_steps, st.R)
            if rec is not None and st.fed_steps and s % st.round_len == 0 and s < st.fed_steps:
                vl = rec.round_start(s)  # val of the round's start model (also the ES value at minibatch 0)
                if use_es and s % per_epoch_fed == 0:
                    val_hist[0].append(vl)
            elif use_es and st.fed_steps and s % per_epoch_fed == 0 and s < st.fed_steps:
                live = [ci for ci in fed if not st.stopped[ci]]
                if live:  # val loss of each live global model at the start of epoch e (minibatch 0)
                    for ci, l in zip(live, self._val_loss(st.glob, live)):
                        val_hist[orig[ci]].append(l)
            st.step(s)
            if rec is not None:
                rec.after_step(s)
            if st.fed_steps and s < st.fed_steps and (s + 1) % st.round_len == 0:
                if rec is not None:
                    rec.round_end(s)
                st.aggregate(epoch_end=(s + 1) % per_epoch_fed == 0)
                if use_es and (s + 1) % per_epoch_fed == 0:
                    e = (s + 1) // per_epoch_fed - 1
                    stops = []
                    for ci in fed:
                        h = val_hist[orig[ci]]
                        if not st.stopped[ci] and e >= PATIENCE and h[e] > h[e - PATIENCE]:
                            epochs_done[orig[ci]] = e + 1
                            stops.append(ci)
                    if stops:
                        st.stop(stops)
            if use_es and spe:
                # singleton epoch ends: Keras EarlyStopping(monitor='val_loss', patience=10, min_delta=0)
                ends = [ci for ci in spe if not st.stopped[ci] and (s + 1) % spe[ci] == 0
                        and (s + 1) // spe[ci] <= epochs]
                if ends:
                    stops = []
                    for ci, l in zip(ends, self._val_loss(st.params, [st.coal_first[c] for c in ends])):
                        e = (s + 1) // spe[ci] - 1
                        o = orig[ci]
                        val_hist[o].append(l)
                        if l < es_best[o]:
                            es_best[o], es_wait[o] = l, 0
                        else:
                            es_wait[o] += 1
                            if es_wait[o] >= PATIENCE:
                                epochs_done[o] = e + 1
                                stops.append(ci)
                    if stops:
                        st.stop(stops)
            if st.stopped.all():
                break
        if rec is not None:
            rec.finish(epochs_done[0])
        glob = st.finalize()
        self.last_es_trace = val_hist
        self.last_models = glob.cpu().numpy() if keep_models else None
        if getattr(eng, "time_test_eval", False):  # bench accounting: the test evaluation's own time
            import time
            import torch
            torch.cuda.synchronize(eng.device)
            t0 = time.perf_counter()
        c_end, _ = self._evaluate(glob, list(range(st.C)), eng.x_test_d, eng.y_test_d)
        correct[orig] = c_end
        if getattr(eng, "time_test_eval", False):
            eng.stats["test_eval_s"] = eng.stats.get("test_eval_s", 0.0) + time.perf_counter() - t0
        return correct / float(eng.y_test_d.numel()), epochs_done

    def run_concurrent(self, parts, epochs):
        """Independent lockstep batches (`parts`: lists of coalitions) trained step by step interleaved, each on
        its own HIP stream, so that their kernels overlap on the device (the CIFAR step's ~0.3 ms kernels leave
        tails and launch gaps a second batch fills).  No early stopping, history or kept models
        (CoalitionEngine.evaluate falls back to run() for those).  A batch the bench's kernel timer samples (the
        profiler set by eng.progress at the batch's start) runs as ONE lockstep batch on the caller's stream: its
        launches are then timed without another stream's kernels overlapping them, and each launch covers the
        whole batch, as in a single-stream run (round 5's parts run "in turn" were still concurrent on the device:
        only their enqueueing was sequential, so every timed launch shared the GPU with the other part's).
        v(S) depends only on (S, seed): every value is the one the same coalition gets in any other batch.
        Returns the test accuracies per part."""
        import torch
        eng = self.eng
        dev = eng.device
        stats = eng.stats
        progress = getattr(eng, "progress", None)
        if progress is not None:  # batch start, as run() reports it (the bench's in-stream timer samples batches)
            geo = [schedule_geometry(eng, coal, epochs)[2] for coal in parts]
            progress(0, max(geo), sum(len(c) for coal in parts for c in coal))
        if eng.profiler is not None:
            flat = [c for coal in parts for c in coal]
            acc, _ = self.run(flat, epochs, False, started=True)
            out, i = [], 0
            for coal in parts:
                out.append(acc[i:i + len(coal)])
                i += len(coal)
            return out
        main = torch.cuda.current_stream(dev)
        # the same side streams for every batch: the caching allocator keeps its blocks per stream, so fresh streams
        # would make every lockstep batch allocate its buffers anew
        pool = getattr(self, "_side_streams", [])
        while len(pool) < len(parts):
            pool.append(torch.cuda.Stream(device=dev))
        self._side_streams = pool
        streams = pool[:len(parts)]
        sts = []
        for coal, sm in zip(parts, streams):
            sm.wait_stream(main)  # the data and anything queued before on the caller's stream
            with torch.cuda.stream(sm):
                sts.append(self.prepare(coal, epochs))
        for s in range(max(st.total_steps for st in sts)):
            for st, sm in zip(sts, streams):
                if s >= st.total_steps:
                    continue
                with torch.cuda.stream(sm):
                    stats["replica_steps"] = stats.get("replica_steps", 0) + st.R
                    stats["replica_steps_live"] = stats.get("replica_steps_live", 0) + int(
                        np.sum(st.kind_host != REP_IDLE))
                    st.step(s)
                    if st.fed_steps and s < st.fed_steps and (s + 1) % st.round_len == 0:
                        st.aggregate(epoch_end=(s + 1) % (eng.minibatch_count * st.round_len) == 0)
        out = []
        for st, sm in zip(sts, streams):
            with torch.cuda.stream(sm):
                glob = st.finalize()
                c_end, _ = self._evaluate(glob, list(range(st.C)), eng.x_test_d, eng.y_test_d)  # syncs sm
            out.append(c_end / float(eng.y_test_d.numel()))
        for sm in streams:
            main.wait_stream(sm)
        self.last_es_trace = [[] for st in sts for _ in range(st.C)]
        return out

    def _final_correct(self, st, cis):
        """Test hits of the final models of stopped coalitions `cis` of batch `st` (a FedAvg coalition's model
        is its coalition row, a singleton's its replica row)."""
        import torch
        rows = [st.params[st.coal_first[ci]] if st.coal_is_single[ci] else st.glob[ci] for ci in cis]
        models = torch.stack(rows).contiguous()
        correct, _ = self._evaluate(models, list(range(len(cis))), self.eng.x_test_d, self.eng.y_test_d)
        return correct

    def _compact(self, st, live):
        """A batch of the live coalitions `live` of `st` continuing where `st` stands: their coalition rows,
        replica rows and optimizer rows gathered in order, the same schedule geometry; `st` is released."""
        import torch
        dev = self.eng.device
        reps = torch.tensor([r for ci in live for r in range(st.coal_first[ci], st.coal_first[ci + 1])],
                            dtype=torch.int64, device=dev)
        resume = {"glob": st.glob.index_select(0, torch.tensor(live, dtype=torch.int64, device=dev)),
                  "params": st.params.index_select(0, reps),
                  "opt": {k: v.index_select(0, reps) for k, v in st.model.opt_state(st).items()},
                  "round_len": st.round_len, "fed_steps": st.fed_steps, "total_steps": st.total_steps}
        coalitions, epochs = [st.coalitions[ci] for ci in live], st.epochs
        st.release()
        return TrainBatch(self.eng, coalitions, epochs, self.lib, resume=resume)

    # --------------------------------------------------------------------------------------------
    def _evaluate(self, params, rows, x, y):
        import torch
        sel = params if rows == list(range(params.shape[0])) else params[torch.tensor(rows, device=self.eng.device)].contiguous()
        return self.eng.model_impl.evaluate(self.eng, sel, x, y)

    def _val_loss(self, params, rows):
        import time
        import torch
        # the stats time the evaluation itself: the training steps the host queued ahead finish first (the
        # loss's host copy below synchronises anyway, so this wait costs no throughput)
        torch.cuda.synchronize(self.eng.device)
        t0 = time.perf_counter()
        _, loss = self._evaluate(params, rows, self.eng.x_val_d, self.eng.y_val_d)  # synchronises (host copy)
        st = self.eng.stats
        st["es_val_s"] = st.get("es_val_s", 0.0) + time.perf_counter() - t0
        st["es_val_evals"] = st.get("es_val_evals", 0) + len(rows)
        return [float(v) for v in loss]


class HistoryRecorder:
    """The learning history of one coalition's training (mplc/mpl_utils.py:11-27 History.history):
    'mpl_model' val_loss / val_accuracy [E, M] of the round-start global model (eval_and_log_model_val_perf,
    called at the start of every round, mplc/multi_partner_learning.py:142-156, 319-320, 363-364) and, per
    partner, the Keras fit history of its round (log_partner_perf, :130-133): 'loss' / 'accuracy' are the
    running training values of the fit (per-sample CE and correct predictions before each update, from
    the head kernel's hstats), 'val_loss' / 'val_accuracy' those of the partner's model after the fit.
    A singleton (SinglePartnerLearning, :238-269) logs its last epoch at [0, 0] and has no 'mpl_model'.
    Unvisited entries keep the reference's initial values (NaN for partners, 0 for the collective model)."""
    METRICS = ("val_accuracy", "val_loss", "loss", "accuracy")

    def __init__(self, trainer, st, epochs, out):
        eng = trainer.eng
        self.trainer, self.st, self.eng = trainer, st, eng
        self.coal = st.coalitions[0]
        self.k = len(self.coal)
        self.M = eng.minibatch_count
        self.mask = sum(1 << p for p in self.coal)
        self.n_val = float(eng.y_val_d.numel())
        self.h = out
        for p in self.coal:
            out[p] = {m: np.full((epochs, self.M), np.nan) for m in self.METRICS}
        if self.k > 1:
            out["mpl_model"] = {"val_accuracy": np.zeros((epochs, self.M)), "val_loss": np.zeros((epochs, self.M))}
        self.acc = np.zeros((self.k, 3))
        self.single_spe = None
        if self.k == 1:
            p = self.coal[0]
            self.single_spe = -(-eng.partner_sizes[p] // eng.batch_sizes[p])
            self.last = None
        self.order_steps = None

    def _val(self, params, rows):
        correct, loss = self.trainer._evaluate(params, rows, self.eng.x_val_d, self.eng.y_val_d)
        return correct / self.n_val, loss

    def round_start(self, s):
        e, m = divmod(s // self.st.round_len, self.M)
        acc, loss = self._val(self.st.glob, [0])
        self.h["mpl_model"]["val_accuracy"][e, m] = acc[0]
        self.h["mpl_model"]["val_loss"][e, m] = loss[0]
        self.acc[:] = 0.0
        if self.st.seq_mode:  # member visiting order and fit lengths of this round
            b = self.eng.bounds
            order = seq_member_order(self.eng.seed, self.mask, self.k, e, m)
            self.order_steps = []
            for mi in order:
                p = self.coal[mi]
                self.order_steps.extend([mi] * (-(-(b[p][m + 1] - b[p][m]) // self.eng.batch_sizes[p])))
        return float(loss[0])

    def after_step(self, s):
        hs = self.st.hstats.cpu().numpy()
        if self.k == 1:
            t = s % self.single_spe
            if t == 0:
                self.acc[:] = 0.0
            self.acc[0] += hs[0]
            if t == self.single_spe - 1 and s // self.single_spe < self.st.epochs:
                self.last = self.acc[0].copy()  # the epoch's running loss / accuracy
            return
        if s >= self.st.fed_steps:
            return
        if self.st.seq_mode:
            t = s % self.st.round_len
            if t < len(self.order_steps):
                self.acc[self.order_steps[t]] += hs[0]
        else:
            self.acc += hs[:self.k]

    def round_end(self, s):
        e, m = divmod(s // self.st.round_len, self.M)
        st = self.st
        if st.seq_mode:
            base = st.snap_row(0)
            acc, loss = self._val(st.snap, [base + mi for mi in range(self.k)])
        else:
            acc, loss = self._val(st.params, list(range(st.coal_first[0], st.coal_first[0] + self.k)))
        for mi, p in enumerate(self.coal):
            h = self.h[p]
            n = self.acc[mi, 2]
            h["val_accuracy"][e, m] = acc[mi]
            h["val_loss"][e, m] = loss[mi]
            h["loss"][e, m] = self.acc[mi, 0] / n if n else np.nan
            h["accuracy"][e, m] = self.acc[mi, 1] / n if n else np.nan

    def finish(self, epochs_done):
        if self.k != 1 or self.last is None:
            return
        p = self.coal[0]
        acc, loss = self._val(self.st.params, [self.st.coal_first[0]])
        h = self.h[p]
        h["val_accuracy"][0, 0], h["val_loss"][0, 0] = acc[0], loss[0]
        h["loss"][0, 0] = self.last[0] / self.last[2]
        h["accuracy"][0, 0] = self.last[1] / self.last[2]
