"""Host hooks of the batched CIFAR10 CNN trainer (csrc/cifar_cnn.hip, include/mplc_hip_cifar.h).

Architecture and optimizer of the reference's Cifar10.generate_new_model (mplc/dataset.py:167-200):
Conv(32,same) Conv(32) Pool Dropout(.25) Conv(64,same) Conv(64) Pool Dropout(.25) Dense(512) Dropout(.5)
Dense(10); categorical CE; RMSprop(learning_rate=1e-4, decay=1e-6) with Keras 2.3.1 defaults rho=0.9,
epsilon=1e-7.  The coalition orchestration (FedAvg rounds with a fresh optimizer per partner fit,
singletons with a persistent one, early stopping, test accuracy) is the model-independent TrainBatch /
CnnBatchTrainer of mplc/cnn.py; this module provides the CIFAR parameter layout, state and launches.
"""
import ctypes

import numpy as np

from . import _native
from .cnn import eval_plan

STRIDE = 1251008
NPARAM = 1250954
WG_SAMPLES = 2
A1, D2, A3, D4, H5 = 32768, 7200, 14400, 2304, 512
IMG_FLOATS = 32 * 32 * 3
DZ4, DZ3, DZ2, DZ1 = 2304, 14400, 7200, 32768  # dz4 / dz2: the pooled gradients (ABI 3)
WT, WPART = 114688, 65664  # MPLC_CIFAR_WT: conv2..conv4 in Winograd form
EVAL_FLOATS = A1 + D2 + A3 + D4 + H5  # per model per evaluated sample

KERNEL_IDS = {"conv1_fwd": 1, "conv2_fwd": 2, "conv3_fwd": 3, "conv4_fwd": 4, "dense5_fwd": 5, "head": 6,
              "dense5_bwd": 7, "conv4_wgrad": 8, "conv4_dgrad": 9, "conv3_wgrad": 10, "conv3_dgrad": 11,
              "conv2_wgrad": 12, "conv2_dgrad": 13, "conv1_wgrad": 14, "rmsprop_small": 15}
# algorithmic FLOPs per sample of each profiled launch (bench roofline): what the kernel's algorithm executes.
# conv2..conv4 run in Winograd form F(2x2,3x3) / F(3x3,2x2): (2x2 output tiles) x 16 transform points x CI x CO
# multiply-adds; conv1 is a direct implicit GEMM.  DIRECT_FLOP_PER_SAMPLE: the direct convolution's count (the
# reference's arithmetic), 2.25x the Winograd count, reported beside it as the equivalent rate.
FLOP_PER_SAMPLE = {"conv1_fwd": 1024 * 32 * 27 * 2, "conv2_fwd": 225 * 16 * 32 * 32 * 2,
                   "conv3_fwd": 64 * 16 * 32 * 64 * 2, "conv4_fwd": 36 * 16 * 64 * 64 * 2,
                   "conv4_dgrad": 64 * 16 * 64 * 64 * 2, "conv3_dgrad": 64 * 16 * 64 * 32 * 2,
                   "conv2_dgrad": 256 * 16 * 32 * 32 * 2, "conv4_wgrad": 36 * 16 * 64 * 64 * 2,
                   "conv3_wgrad": 64 * 16 * 32 * 64 * 2, "conv2_wgrad": 225 * 16 * 32 * 32 * 2,
                   "conv1_wgrad": 1024 * 32 * 27 * 2}
DIRECT_FLOP_PER_SAMPLE = {"conv1_fwd": 1024 * 32 * 27 * 2, "conv2_fwd": 900 * 32 * 288 * 2,
                          "conv3_fwd": 225 * 64 * 288 * 2, "conv4_fwd": 144 * 64 * 576 * 2,
                          "conv4_dgrad": 144 * 64 * 576 * 2, "conv3_dgrad": 225 * 32 * 576 * 2,
                          "conv2_dgrad": 900 * 32 * 288 * 2, "conv4_wgrad": 144 * 64 * 576 * 2,
                          "conv3_wgrad": 225 * 64 * 288 * 2, "conv2_wgrad": 900 * 32 * 288 * 2,
                          "conv1_wgrad": 1024 * 32 * 27 * 2}

# conv1's algorithmic HBM bytes per sample: K = 27 (3 input channels) gives it 2 x 27 = 54 flops per output value,
# 12.3 flops per byte of its compulsory traffic, under the fp32 MFMA / HBM ridge (157.3 / 8 = 19.7): its roofline is
# HBM.  fwd: the image read (32 x 32 x 3 fp32) and a1 written (32 x 32 x 32 fp32); wgrad: the image and dz1 read
# (dz1 = conv2's data gradient through relu', written by conv2_dgrad), the per-group dW1 partials (27 x 32 + 32
# floats per MPLC_CIFAR_WG_SAMPLES samples) are not counted.
BYTES_PER_SAMPLE = {"conv1_fwd": 4 * (IMG_FLOATS + A1), "conv1_wgrad": 4 * (IMG_FLOATS + DZ1)}

# Compulsory HBM bytes of EVERY training launch (set beside the FETCH + WRITE counters of the same
# launches, scripts/pmc_traffic.py): each tensor a launch must read or write, once.  Per trained sample the
# activations / gradients (fp32, the pool / dropout / ReLU codes one byte per element); per active replica-step the
# Winograd weights the convolutions read (U, 16 x CI x CO: the data gradients' rotated form has the same size) and the
# head's W6 / b6 RMSprop update; per weight-gradient split (WG_SAMPLES samples) the partial row it writes, and
# rmsprop_small reads those partials and reads and writes W1..b4 and their accumulators.  dense5_fwd / dense5_bwd
# keep their exact schedule-dependent count (algorithmic_units).  The stores of the dz / code tensors that the next
# launch reads are counted on both sides, as they cross HBM twice.
_F = 4
_U2, _U3, _U4 = 16 * 32 * 32, 16 * 32 * 64, 16 * 64 * 64
_W6 = H5 * 10 + 10
_SMALL = 65664  # W1..b4 (the params prefix rmsprop_small updates; = WPART)
SAMPLE_IO = {"conv1_fwd": _F * (IMG_FLOATS + A1), "conv2_fwd": _F * (A1 + D2) + D2, "conv3_fwd": _F * (D2 + A3),
             "conv4_fwd": _F * (A3 + D4) + D4, "head": _F * 2 * H5 + H5,
             "conv4_wgrad": _F * (A3 + DZ4) + D4, "conv4_dgrad": _F * (DZ4 + A3 + DZ3) + D4,
             "conv3_wgrad": _F * (D2 + DZ3), "conv3_dgrad": _F * (DZ3 + DZ2) + D2,
             "conv2_wgrad": _F * (A1 + DZ2) + D2, "conv2_dgrad": _F * (DZ2 + A1 + DZ1) + D2,
             "conv1_wgrad": _F * (IMG_FLOATS + DZ1)}
REPLICA_STEP_IO = {"conv2_fwd": _F * _U2, "conv3_fwd": _F * _U3, "conv4_fwd": _F * _U4, "conv4_dgrad": _F * _U4,
                   "conv3_dgrad": _F * _U3, "conv2_dgrad": _F * _U2, "head": _F * 4 * _W6,
                   "rmsprop_small": _F * 4 * _SMALL}
SPLIT_IO = {"conv4_wgrad": _F * (36864 + 64), "conv3_wgrad": _F * (18432 + 64), "conv2_wgrad": _F * (9216 + 32),
            "conv1_wgrad": _F * (864 + 32), "rmsprop_small": _F * _SMALL}
# the evaluation's forward (mplc_cifar_evaluate: no dropout codes; weights per model and sample chunk)
EVAL_SAMPLE_IO = {"conv1_fwd": _F * (IMG_FLOATS + A1), "conv2_fwd": _F * (A1 + D2), "conv3_fwd": _F * (D2 + A3),
                  "conv4_fwd": _F * (A3 + D4), "dense5_fwd": _F * (D4 + H5)}
EVAL_CHUNK_IO = {"conv2_fwd": _F * _U2, "conv3_fwd": _F * _U3, "conv4_fwd": _F * _U4, "dense5_fwd": _F * (D4 * H5 + H5)}
# rocprofv3 kernel names (template instances, csrc/cifar_cnn.hip CONV* macros) -> the step's launch names
KERNEL_NAME_PREFIX = (("conv1_fwd_kernel", "conv1_fwd"), ("conv_kernel<32, 32, 3, 32", "conv1_fwd"),
                      ("wino_wl_kernel<32, 32, 32, 32", "conv2_fwd"),
                      ("wino_kernel<15, 15, 32, 64", "conv3_fwd"), ("wino_kernel<15, 15, 64, 64", "conv4_fwd"),
                      ("dense5_fwd16_kernel", "dense5_fwd"), ("dense5_fwd_kernel", "dense5_fwd"),
                      ("head_kernel", "head"), ("dense5_bwd_kernel", "dense5_bwd"),
                      ("wino_wgrad_kernel<15, 15, 64, 64", "conv4_wgrad"), ("wino_kernel<13, 13, 64, 64", "conv4_dgrad"),
                      ("wino_wgrad_kernel<15, 15, 32, 64", "conv3_wgrad"), ("wino_kernel<15, 15, 64, 32", "conv3_dgrad"),
                      ("wino_wgrad_kernel<32, 32, 32, 32", "conv2_wgrad"), ("wino_wl_kernel<30, 30, 32, 32", "conv2_dgrad"),
                      ("wgrad_kernel<32, 32, 3, 32", "conv1_wgrad"), ("rmsprop_small_kernel", "rmsprop_small"),
                      ("eval_head_kernel", "eval_head"), ("wino_u_kernel", "wino_u"), ("schedule_kernel", "schedule"))


def launch_name(kernel):
    """The step's launch name of a rocprofv3 kernel name (None: not a CIFAR trainer kernel)."""
    k = kernel.replace("(anonymous namespace)::", "").replace("void ", "").strip()
    for prefix, name in KERNEL_NAME_PREFIX:
        if k.startswith(prefix):
            return name
    return None


def compulsory_bytes(stash, evals):
    """Compulsory HBM bytes and launches per kernel of the stashed training steps [(cnt, opt_t, w5src)] and the
    evaluations [(n_models, samples, chunks)] of a run (StashOnly): {name: {"bytes": total, "launches": n}}.  The
    forward kernels' totals include the evaluation launches, which rocprofv3 reports under the same names."""
    import torch
    out = {k: {"bytes": 0.0, "launches": 0} for k in list(SAMPLE_IO) + ["dense5_fwd", "dense5_bwd", "rmsprop_small"]}
    u = CifarModel.algorithmic_units(stash)
    for cnt, _at, _src in stash:
        c = cnt.to(torch.float64)
        n, reps = float(c.sum()), float((c > 0).sum())
        splits = float(torch.ceil(c / WG_SAMPLES).sum())
        for k in out:
            out[k]["launches"] += 1
            out[k]["bytes"] += SAMPLE_IO.get(k, 0) * n + REPLICA_STEP_IO.get(k, 0) * reps + SPLIT_IO.get(k, 0) * splits
    out["dense5_fwd"]["bytes"] += u.get("dense5_fwd_bytes", 0.0)
    out["dense5_bwd"]["bytes"] += u.get("dense5_bwd_bytes", 0.0)
    for n_models, samples, chunks in evals:
        for k in EVAL_SAMPLE_IO:
            out[k]["launches"] += chunks
            out[k]["bytes"] += EVAL_SAMPLE_IO[k] * n_models * samples + EVAL_CHUNK_IO.get(k, 0) * n_models * chunks
    return out


class CifarTrainT(ctypes.Structure):
    _fields_ = ([("n_rep", ctypes.c_int32), ("bmax", ctypes.c_int32), ("wg_splits", ctypes.c_int32),
                 ("pad0", ctypes.c_int32), ("step", ctypes.c_int32), ("minibatch_count", ctypes.c_int32),
                 ("round_len", ctypes.c_int32), ("epochs", ctypes.c_int32)]
                + [(n, ctypes.c_void_p) for n in ("reps", "rows", "splits", "seq", "x", "labels", "params", "rms", "idx",
                                                   "cnt", "opt_t", "drop_key", "a1", "d2", "code2", "a3", "d4",
                                                   "code4", "d5", "code5", "dh5", "dz4", "dz3", "dz2", "dz1", "wt",
                                                   "wpart")]
                + [(n, ctypes.c_float) for n in ("lr", "rho", "one_minus_rho", "decay", "eps")]
                + [("prof_kernel", ctypes.c_int32), ("prof_begin", ctypes.c_void_p), ("prof_end", ctypes.c_void_p),
                   ("hstats", ctypes.c_void_p), ("glob", ctypes.c_void_p), ("rep_glob", ctypes.c_void_p),
                   ("w5src", ctypes.c_void_p)])


_BOUND = False


def _bind():
    global _BOUND
    if _BOUND:
        return
    _native.register("mplc_cifar_train_step", ctypes.c_int, [ctypes.POINTER(CifarTrainT), ctypes.c_void_p])
    lib = _native.lib()
    global WG_SAMPLES
    WG_SAMPLES = int(lib.mplc_cifar_wgrad_split_samples())  # the library's weight-gradient split size
    _native.check_layout(lib.mplc_cifar_layout, layout_items(), "CIFAR10 CNN")
    _BOUND = True


def layout_items():
    """The host's view of every MPLC_CIFAR_Q_* layout item (include/mplc_hip_cifar.h): name -> (query id, value)."""
    return {"STRIDE": (0, STRIDE), "NPARAM": (1, NPARAM), "A1": (2, A1), "D2": (3, D2), "A3": (4, A3), "D4": (5, D4),
            "H5": (6, H5), "DZ4": (7, DZ4), "DZ3": (8, DZ3), "DZ2": (9, DZ2), "DZ1": (10, DZ1), "WT": (11, WT),
            "WPART": (12, WPART), "WG_SAMPLES": (13, WG_SAMPLES), "TRAIN_T_BYTES": (14, ctypes.sizeof(CifarTrainT))}


class CifarModel:
    """Model hooks (see mplc.cnn.MnistModel) for the CIFAR10 CNN."""
    name = "cifar10_cnn"
    EVAL_SAMPLE_BYTES, EVAL_MODEL_BYTES = EVAL_FLOATS * 4, WT * 4  # evaluation workspace (mplc_cifar_evaluate)
    STRIDE, NPARAM = STRIDE, NPARAM
    # Keras get_weights() order (mplc/dataset.py:170-190): (offset in a model row, shape)
    KERAS_LAYERS = ((0, (3, 3, 3, 32)), (896, (32,)), (960, (3, 3, 32, 32)), (10176, (32,)), (10240, (3, 3, 32, 64)),
                    (28672, (64,)), (28736, (3, 3, 64, 64)), (65600, (64,)), (65664, (2304, 512)), (1245312, (512,)),
                    (1245824, (512, 10)), (1250944, (10,)))
    KERNEL_IDS = KERNEL_IDS
    input_shape = (32, 32, 3)
    # FedAvg aggregation leaves W5 (94 % of the parameters) out of the broadcast: a round's first step reads
    # it from the coalition row (mplc_cifar_train_t.glob, mplc_fedavg_aggregate_bcast_skip)
    BCAST_SKIP = (KERAS_LAYERS[8][0], KERAS_LAYERS[9][0])
    # Keras 2.3.1 RMSprop(learning_rate=0.0001, decay=1e-6): rho 0.9, epsilon K.epsilon() = 1e-7
    lr, rho, decay, eps = 1e-4, 0.9, 1e-6, 1e-7

    def __init__(self):
        _bind()
        self.lib = _native.lib()

    def replica_bytes(self, bmax):
        slot = 4 * (A1 + D2 + A3 + D4 + 2 * H5 + DZ4 + DZ3 + DZ2 + DZ1) + (D2 + D4 + H5) + 4
        splits = (bmax + WG_SAMPLES - 1) // WG_SAMPLES
        return 2 * STRIDE * 4 + bmax * slot + WT * 4 + splits * WPART * 4 + 24

    def init_params(self, glob, keys, stream):
        _native.check(self.lib.mplc_cifar_init_params(_native.ptr(glob), STRIDE, _native.ptr(keys), glob.shape[0],
                                                      stream), "mplc_cifar_init_params")

    def alloc(self, st):
        import torch
        eng, dev, R, B = st.eng, st.dev, st.R, st.bmax
        f32 = dict(dtype=torch.float32, device=dev)
        u8 = dict(dtype=torch.uint8, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        splits = (B + WG_SAMPLES - 1) // WG_SAMPLES
        opt = getattr(st, "resume_opt", None)  # a compacted batch continues its replicas' accumulators
        st.rms = opt["rms"] if opt else torch.zeros((R, STRIDE), **f32)
        st.ws = dict(
            idx=torch.empty((R, B), **i32), cnt=torch.empty(R, **i32), opt_t=torch.empty(R, **i32),
            drop_key=torch.empty(R, dtype=torch.int64, device=dev),
            a1=torch.empty((R, B, A1), **f32), d2=torch.empty((R, B, D2), **f32), code2=torch.empty((R, B, D2), **u8),
            a3=torch.empty((R, B, A3), **f32), d4=torch.empty((R, B, D4), **f32), code4=torch.empty((R, B, D4), **u8),
            d5=torch.empty((R, B, H5), **f32), code5=torch.empty((R, B, H5), **u8), dh5=torch.empty((R, B, H5), **f32),
            dz4=torch.empty((R, B, DZ4), **f32), dz3=torch.empty((R, B, DZ3), **f32),
            dz2=torch.empty((R, B, DZ2), **f32), dz1=torch.empty((R, B, DZ1), **f32),
            wt=torch.empty((R, WT), **f32), wpart=torch.empty((R, splits, WPART), **f32), w5src=torch.empty(R, **i32))
        t = CifarTrainT()
        t.n_rep, t.bmax, t.wg_splits = R, B, splits
        t.minibatch_count, t.round_len, t.epochs = eng.minibatch_count, st.round_len, st.epochs
        t.reps, t.rows, t.splits = st.rep_t.data_ptr(), eng.rows_d.data_ptr(), eng.splits_d.data_ptr()
        t.seq = st.seq_t.data_ptr() if st.seq_t is not None else None
        t.x, t.labels = eng.x_train_d.data_ptr(), eng.y_train_d.data_ptr()
        t.params, t.rms = st.params.data_ptr(), st.rms.data_ptr()
        for k, v in st.ws.items():
            setattr(t, k, v.data_ptr())
        t.lr, t.rho, t.decay, t.eps = self.lr, self.rho, self.decay, self.eps
        t.one_minus_rho = float(np.float32(1.0 - self.rho))  # Keras: (1. - rho) on the Python double
        if not st.seq_mode:  # FedAvg rounds start from the coalition row (W5 is not broadcast)
            t.glob, t.rep_glob = st.glob.data_ptr(), st.src_map.data_ptr()
        st.t = t

    def free(self, st):
        st.rms = None

    @staticmethod
    def opt_state(st):
        """The per-replica optimizer rows of a TrainBatch (RMSprop accumulators)."""
        return {"rms": st.rms}

    def step(self, st, s, prof):
        st.t.step = s
        if prof is not None:
            if prof.all:
                prof.bind(self.KERNEL_IDS)
            ev0, ev1 = prof.pair()
            st.t.prof_kernel = -1 if prof.all else self.KERNEL_IDS[prof.kernel]  # -1: MPLC_PROF_ALL
            st.t.prof_begin, st.t.prof_end = ev0, ev1
        else:
            st.t.prof_kernel, st.t.prof_begin, st.t.prof_end = 0, None, None
        _native.check(self.lib.mplc_cifar_train_step(ctypes.byref(st.t), st.stream), "mplc_cifar_train_step")
        if prof is not None and prof.want_stash:
            prof.stash_step(st.ws["cnt"], st.ws["opt_t"], st.ws["w5src"])

    @staticmethod
    def algorithmic_units(stash):
        """Algorithmic work of the timed steps from their stashed schedules [(cnt, opt_t, w5src)]: samples (the
        convolutions' unit) and the HBM bytes of the two W5 kernels (csrc/cifar_cnn.hip):
          dense5_fwd: W5 read; per sample the d4 row read, the h5 row written with its code byte;
          dense5_bwd: W5 read and written, the RMSprop accumulator written (and read unless the optimizer is
                      fresh, t = 1); per sample d4, its code byte and dh5 read, the POOLED dz4 written (one
                      float per pooled element since round 4; rounds 3-4 counted 4 window pixels, 1.5 % more).
        A FedAvg round's first step reads W5 from the coalition row (w5src >= 0), shared by the coalition's
        replicas: counted once per coalition."""
        import torch
        w5 = float(D4 * H5 * 4)
        samples = d5b = d5f = 0.0
        for cnt, at, src in stash:
            cnt = cnt.to(torch.float64)
            act = (cnt > 0).to(torch.float64)
            shared = src >= 0
            n_shared_rows = float(torch.unique(src[shared & (cnt > 0)]).numel())
            own = (~shared).to(torch.float64)
            acc_rd = (at > 1).to(torch.float64)
            d5b += float((act * (w5 * (own + 2.0 + acc_rd)) + cnt * float(D4 * 4 + D4 + H5 * 4 + D4 * 4)).sum())
            d5f += float((act * w5 * own + cnt * float(D4 * 4 + H5 * 4 + H5)).sum())
            d5b += n_shared_rows * w5
            d5f += n_shared_rows * w5
            samples += float(cnt.sum())
        return {"samples": samples, "dense5_bwd_bytes": d5b, "dense5_fwd_bytes": d5f}

    def evaluate(self, eng, sel, x, y):
        import torch
        dev = eng.device
        stream = _native.stream_handle(dev)
        n = int(y.numel())
        C = sel.shape[0]
        # the workspace also holds every model's Winograd weights (WT floats per model,
        # mplc_cifar_eval_workspace_floats); cnn.eval_plan keeps the loss sums independent of C
        chunk, group = eval_plan(n, C, self.EVAL_SAMPLE_BYTES, self.EVAL_MODEL_BYTES, eng.eval_budget_bytes)
        ws = torch.empty(int(self.lib.mplc_cifar_eval_workspace_floats(group, chunk)), dtype=torch.float32, device=dev)
        correct = torch.zeros(C, dtype=torch.int32, device=dev)
        loss = torch.zeros(C, dtype=torch.float64, device=dev)
        prof = eng.profiler
        for g0 in range(0, C, group):
            g = min(group, C - g0)
            if prof is not None and hasattr(prof, "stash_eval"):  # (models, samples, chunks) of this launch group
                prof.stash_eval(g, n, -(-n // chunk))
            _native.check(self.lib.mplc_cifar_evaluate(_native.ptr(sel[g0:g0 + g]), STRIDE, g, _native.ptr(x),
                                                       _native.ptr(y), n, chunk, _native.ptr(ws),
                                                       _native.ptr(correct[g0:g0 + g]), _native.ptr(loss[g0:g0 + g]),
                                                       stream), "mplc_cifar_evaluate")
        return correct.cpu().numpy().astype(np.float64), loss.cpu().numpy() / n
