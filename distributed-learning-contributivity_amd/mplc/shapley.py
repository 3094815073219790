"""Exact Shapley aggregation on the MI355X (host side of csrc/shapley.hip).

Public surface:
  shapley_value(partners_count, char_func_list)  - drop-in for mplc/contributivity.py:1210-1253
  ShapleyAggregator(n).run(V_device)             - bitmask table already resident in HBM (bench / engine)
  ShapleyAggregator(n).partial(V_shard, begin)   - range-sharded partial sums for the multi-GPU path
  ShapleyAggregator.finalize(partial)            - SV from (all-reduced) partial sums
"""
import numpy as np

from . import _native
from .coalitions import combination_list_to_bitmask

SPAN = 65536  # masks per block of the n >= 16 kernel; shard boundaries must be multiples of it


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("MI355X (HIP) device required: the MPLC engine has no CPU fallback")
    return torch


class ShapleyAggregator:
    """Reusable device workspace for one n (the library itself allocates nothing)."""

    def __init__(self, n, device=None, count=None):
        torch = _torch()
        if not 1 <= n <= 40:
            raise ValueError("partners_count must be in [1, 40]")
        self.n = n
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.lib = _native.lib()
        count = (1 << n) if count is None else int(count)
        self.ws_bytes = int(self.lib.mplc_shapley_workspace_bytes(n, count)) + 16 * (n + 1)
        self.ws = torch.empty(max(self.ws_bytes, 16), dtype=torch.uint8, device=self.device)
        self.partial_buf = torch.empty(2 * (n + 1), dtype=torch.float64, device=self.device)
        self.sv = torch.empty(n, dtype=torch.float64, device=self.device)

    def run(self, V):
        """V: float64 CUDA tensor of 2^n entries in bitmask order.  Returns the SV tensor (device, async)."""
        if V.dtype != _torch().float64 or V.numel() != (1 << self.n) or not V.is_contiguous():
            raise ValueError("V must be a float64 device tensor with 2^n entries")
        st = self.lib.mplc_shapley_exact(_native.ptr(V), self.n, _native.ptr(self.sv), _native.ptr(self.ws),
                                         self.ws_bytes, _native.stream_handle(self.device))
        _native.check(st, "mplc_shapley_exact")
        return self.sv

    def partial(self, V_shard, mask_begin):
        """Partial sums (2(n+1) float64, device) over masks [mask_begin, mask_begin + len(V_shard))."""
        count = V_shard.numel()
        need = int(self.lib.mplc_shapley_workspace_bytes(self.n, count))
        if need + 16 * (self.n + 1) > self.ws_bytes:
            raise RuntimeError("workspace too small for this shard")
        st = self.lib.mplc_shapley_partial(_native.ptr(V_shard), int(mask_begin), int(count), self.n,
                                           _native.ptr(self.partial_buf), _native.ptr(self.ws), self.ws_bytes,
                                           _native.stream_handle(self.device))
        _native.check(st, "mplc_shapley_partial")
        return self.partial_buf

    def finalize(self, partial):
        st = self.lib.mplc_shapley_finalize(_native.ptr(partial), self.n, _native.ptr(self.sv),
                                            _native.stream_handle(self.device))
        _native.check(st, "mplc_shapley_finalize")
        return self.sv


def shard_range(n, rank, world_size):
    """[begin, end) mask range of `rank` for the range-sharded aggregation (block-aligned for n >= 16)."""
    total = 1 << n
    if n < 16:
        return (0, total) if rank == 0 else (0, 0)
    nblocks = total // SPAN
    b0 = nblocks * rank // world_size
    b1 = nblocks * (rank + 1) // world_size
    return b0 * SPAN, b1 * SPAN


def sharded_shapley(V, n, rank, world_size):
    """SV of a full bitmask table that every rank holds (the all-reduced v(S) of the engine's sharded
    evaluation): each rank reduces its block-aligned mask range [shard_range) once, the 2(n+1) partial sums
    are all_reduced (RCCL on the GPUs; through host memory for a gloo rehearsal), and every rank finalizes the
    same SV.  The sums are linear in V, so the result equals the one-pass kernel's to rounding
    (1e-12 relative, tests/test_shapley_gpu.py)."""
    import torch.distributed as dist
    torch = _torch()
    begin, end = shard_range(n, rank, world_size)
    agg = ShapleyAggregator(n, device=V.device, count=max(end - begin, SPAN))
    if end > begin:
        part = agg.partial(V[begin:end], begin)
    else:
        part = agg.partial_buf.zero_()
    if dist.get_backend() == "nccl":
        dist.all_reduce(part)
    else:
        host = part.cpu()
        dist.all_reduce(host)
        part.copy_(host)
    return agg.finalize(part).cpu().numpy()


def shapley_from_table(V, n, sharded=False):
    """SV (numpy float64, length n) of a bitmask-ordered table given as numpy array or device tensor.

    sharded=True is a COLLECTIVE: under torch.distributed with n >= 16 every rank must call it with the same
    table, which is then reduced range-sharded across the ranks (sharded_shapley).  The default is local, as
    the reference's pure function (a caller on one rank, e.g. post-processing on rank 0, must not block)."""
    from .parallel import world
    torch = _torch()
    if isinstance(V, np.ndarray):
        V = torch.from_numpy(np.ascontiguousarray(V, dtype=np.float64)).cuda()
    rank, ws = world()
    if sharded and ws > 1 and n >= 16:
        return sharded_shapley(V, n, rank, ws)
    agg = ShapleyAggregator(n, device=V.device)
    return agg.run(V).cpu().numpy()


def shapley_value(partners_count, char_func_list, sharded=False):
    """Drop-in for the reference ``shapley_value`` (mplc/contributivity.py:1210-1253).

    char_func_list: v(S) of the 2^n - 1 non-empty coalitions in combination order (as built by
    compute_SV, mplc/contributivity.py:149-158).  Returns a list of n floats.
    The reference calls quit() for n == 0 (mplc/contributivity.py:1214-1216); this raises ValueError.
    sharded=True (compute_SV, where every rank holds the all-reduced table): a collective, see
    shapley_from_table; the default computes locally like the reference's pure function.
    """
    n = int(partners_count)
    if n == 0:
        raise ValueError("No players")
    table = combination_list_to_bitmask(n, char_func_list)
    return [float(x) for x in shapley_from_table(table, n, sharded=sharded)]
