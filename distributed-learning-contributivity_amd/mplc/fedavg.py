"""FedAvg weighted partner aggregation (host side of csrc/fedavg.hip).

Mirrors mplc/mpl_utils.py:82-115: the aggregation weights of UniformAggregator ([1/P]*P) and
DataVolumeAggregator (partner sizes / sum), and Aggregator.aggregate_model_weights' np.average
(axis=0, weights=w) in float64 stored back as float32.  The device kernel is bit-identical to numpy.
"""
import numpy as np

from . import _native

AGGREGATION_SCHEMES = ("uniform", "data-volume")


def aggregation_weights(sizes, scheme="data-volume"):
    """Per-partner weights exactly as the reference aggregators build them, and np.average's scale
    (wgt.sum(axis=0) on the broadcast weights, mplc/mpl_utils.py:97-99 -> numpy.average)."""
    P = len(sizes)
    if scheme == "uniform":               # mplc/mpl_utils.py:105-108
        w = [1 / P] * P
    elif scheme == "data-volume":         # mplc/mpl_utils.py:111-115
        w = np.asarray(list(sizes)) / np.sum(list(sizes))
    else:
        raise ValueError(f"aggregation approach '{scheme}' is not a valid approach. ")
    wgt = np.asarray(w, dtype=np.float64).reshape(P, 1)
    scl = float(wgt.sum(axis=0)[0])
    if scl == 0.0:
        raise ZeroDivisionError("Weights sum to zero, can't be normalized")
    return [float(x) for x in np.asarray(w, dtype=np.float64)], scl


def fedavg_aggregate(x, groups, sizes, scheme="data-volume", out=None, broadcast=False):
    """Aggregate replica rows of `x` ([R, n_param] float32 CUDA tensor, or a one-element list of it).

    groups: per coalition, the list of its replica row indices (must be contiguous, ascending);
    sizes: per coalition, the partner data volumes in the same order.
    Returns out [C, n_param] float32 (device).  broadcast=True also writes the result into every
    replica row (start of the next FedAvg round)."""
    import torch
    if isinstance(x, (list, tuple)):
        x = x[0]
    if x.dtype != torch.float32 or x.dim() != 2 or not x.is_cuda:
        raise ValueError("x must be a [R, n_param] float32 CUDA tensor")
    C = len(groups)
    first = [0] * (C + 1)
    ws, scales = [], []
    for c, (g, sz) in enumerate(zip(groups, sizes)):
        if list(g) != list(range(g[0], g[0] + len(g))):
            raise ValueError("replicas of a coalition must be contiguous rows")
        if c > 0 and g[0] != first[c]:
            raise ValueError("coalition groups must tile the replica rows in order")
        first[c] = g[0]
        first[c + 1] = g[0] + len(g)
        w, scl = aggregation_weights(sz, scheme)
        ws.extend(w)
        scales.append(scl)
    dev = x.device
    first_t = torch.tensor(first, dtype=torch.int32, device=dev)
    w_t = torch.zeros(x.shape[0], dtype=torch.float64)
    w_t[first[0]:first[0] + len(ws)] = torch.tensor(ws, dtype=torch.float64)
    w_t = w_t.to(dev)
    scale_t = torch.tensor(scales, dtype=torch.float64, device=dev)
    if out is None:
        out = torch.empty((C, x.shape[1]), dtype=torch.float32, device=dev)
    st = _native.lib().mplc_fedavg_aggregate(_native.ptr(x), x.stride(0), _native.ptr(first_t), _native.ptr(w_t),
                                             _native.ptr(scale_t), C, x.shape[1], _native.ptr(out), out.stride(0),
                                             1 if broadcast else 0, _native.stream_handle(dev))
    _native.check(st, "mplc_fedavg_aggregate")
    return out
