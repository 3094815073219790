"""Monte-Carlo Shapley on the MI355X: truncated permutation walks over a dense bitmask v(S) table
(csrc/mc_shapley.hip, include/mplc_hip.h mplc_tmc_*).

Three uses:
  - VTable: the device copy of the coalition values known so far (NaN = not evaluated), bitmask order.
  - wave_frontier: walk a wave of permutations on device with the reference's truncation test and return
    the unknown prefixes they need next (Contributivity's TMCS/ITMCS batch planner).
  - truncated_mc_table: the reference's truncated_MC / interpol_TMC loop (mplc/contributivity.py:195-322)
    on a fully known table - rows from the device walk, the sequential stopping rule and moments in numpy
    exactly as the reference (bit-identical on the reference goldens, tests/test_mc_gpu.py).
  - tmc_moments: fixed-budget form for large tables (sum / sum of squares per partner reduced on device).
"""
import numpy as np
from scipy.stats import norm

from . import _native

MAX_N = 30


def _torch():
    import torch
    return torch


class VTable:
    """Dense fp64 v(S) table on device: 2^n entries, NaN = unknown, V[0] = 0."""

    def __init__(self, n, device=None):
        torch = _torch()
        if not 1 <= n <= MAX_N:
            raise ValueError(f"dense table supports 1 <= n <= {MAX_N}")
        self.n = n
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.V = torch.full((1 << n,), float("nan"), dtype=torch.float64, device=self.device)
        self.V[0] = 0.0
        self.known = set()

    @staticmethod
    def mask(key):
        m = 0
        for i in key:
            m |= 1 << int(i)
        return m

    def update(self, values):
        """values: {sorted tuple of partner ids: v}; uploads the entries not on the device yet."""
        torch = _torch()
        new = [(self.mask(k), float(v)) for k, v in values.items() if len(k) and k not in self.known]
        if not new:
            return
        idx = torch.tensor([m for m, _ in new], dtype=torch.int64, device=self.device)
        val = torch.tensor([v for _, v in new], dtype=torch.float64, device=self.device)
        self.V.index_put_((idx,), val)
        self.known.update(k for k, v in values.items() if len(k))

    @classmethod
    def from_array(cls, V, device=None):
        torch = _torch()
        V = np.asarray(V, dtype=np.float64)
        n = int(V.size).bit_length() - 1
        if V.size != 1 << n:
            raise ValueError("table length must be a power of two")
        t = cls.__new__(cls)
        t.n = n
        t.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        t.V = torch.from_numpy(V.copy()).to(t.device)
        t.known = None
        return t


def tmc_walk(table, perms, v_all, truncation, interpolate=False, sizes=None):
    """Device walk of each permutation (rows [K][n] fp64, status [K] int32, need [K] uint64 masks)."""
    torch = _torch()
    perms = np.ascontiguousarray(perms, dtype=np.uint8)
    K, n = perms.shape
    if n != table.n:
        raise ValueError("permutation length does not match the table")
    dev = table.device
    p_d = torch.from_numpy(perms).to(dev)
    rows = torch.empty((K, n), dtype=torch.float64, device=dev)
    status = torch.empty(K, dtype=torch.int32, device=dev)
    need = torch.empty(K, dtype=torch.int64, device=dev)
    sz = torch.tensor(np.asarray(sizes, dtype=np.float64), device=dev) if sizes is not None else None
    _native.check(_native.lib().mplc_tmc_walk(_native.ptr(table.V), n, _native.ptr(p_d), K, float(v_all),
                                              float(truncation), int(bool(interpolate)), _native.ptr(sz),
                                              _native.ptr(rows), _native.ptr(status), _native.ptr(need),
                                              _native.stream_handle(dev)), "mplc_tmc_walk")
    return rows.cpu().numpy(), status.cpu().numpy(), need.cpu().numpy().view(np.uint64)


def mask_to_key(mask):
    mask = int(mask)
    return tuple(i for i in range(mask.bit_length()) if (mask >> i) & 1)


def size_predictor(known, n, v_all):
    """v(S) predicted from |S| alone (the speculative planner's truncation model): per size the mean and standard
    deviation of the known values of that size, linear in between, v_all at n.  known: iterable of (key, value).
    Returns (mean[n + 1], sd[n + 1])."""
    vals = [[] for _ in range(n + 1)]
    for k, v in known:
        if 0 < len(k) < n:
            vals[len(k)].append(v)
    vals[n] = [v_all]
    xs = [s for s in range(1, n + 1) if vals[s]]
    mean = np.interp(np.arange(n + 1), xs, [float(np.mean(vals[s])) for s in xs])
    # a size's own spread once it has enough values, else the spread of everything known (never overconfident:
    # an underestimated spread makes the planner speculate past truncations it did not expect)
    pooled = [v for s in range(1, n) for v in vals[s]]
    prior = float(np.std(pooled)) if len(pooled) > 1 else 0.1
    sx = [s for s in range(1, n) if len(vals[s]) >= 10]
    sd = np.interp(np.arange(n + 1), sx, [float(np.std(vals[s])) for s in sx]) if sx else np.full(n + 1, prior)
    sd = np.where([len(vals[s]) >= 10 for s in range(n + 1)], sd, np.maximum(sd, prior))
    return mean, np.maximum(sd, 0.005)


def _p_continue(v, mean, sd, v_all, truncation):
    """Probability that a walk continues past a prefix (its truncation test |v_all - v(prefix)| < truncation does
    not fire): exact for a known value v, else with v ~ N(mean, sd)."""
    if v is not None:
        return 0.0 if abs(v_all - v) < truncation else 1.0
    from scipy.stats import norm
    hit = norm.cdf((v_all + truncation - mean) / sd) - norm.cdf((v_all - truncation - mean) / sd)
    return float(1.0 - hit)


def plan_frontier(perms, stop, value, pred, v_all, truncation, target_replicas, overhead_replicas=16.0):
    """The coalitions to train for one frontier step of a wave of truncated permutation walks
    (mplc/contributivity.py:215-246: a walk needs v(perm[:j+1]) while |v_all - v(perm[:j])| >= truncation).

    perms [K][n]; stop[k] = position j of walk k's first unknown prefix perm[:j+1] (n: the walk is complete).
    Every first unknown prefix is REQUIRED.  Deeper prefixes of the same walks are added as SPECULATION, most
    probable first: the walk reaches perm[:j+2] only if its truncation test does not fire on perm[:j+1] - certain
    when that value is known, else modelled from the known values of the same size (pred = size_predictor).  Each
    speculative coalition S that the walks then do not need costs |S| replica-trainings; each frontier step saved
    costs a lockstep batch's fixed overhead, about `overhead_replicas` replica-trainings (CIFAR10 on one MI355X:
    59 ms per batch vs 3.5 ms per replica, scripts/sim_tmcs_planning.py).  So speculation stops once the expected
    waste sum (1 - p) |S| would exceed that overhead, or the batch holds `target_replicas` replicas.  In the bulk of
    a wave (many walks, a level is worth many batches' overhead) little is speculated; in its tail (few walks)
    whole chains are.  Speculation never changes a result (v(S) is a function of (S, seed) only, and the
    sequential loop still decides what it asks for).  value(key) -> known v or None.
    Returns (keys, number of required keys); keys are sorted tuples."""
    import heapq
    perms = np.asarray(perms)
    K, n = perms.shape
    mean, sd = pred
    chosen = {}
    replicas = 0
    heap = []  # (-p_reach of the chain's next prefix, walk, position of the last chosen prefix)
    for k in range(K):
        j = int(stop[k])
        if j >= n:
            continue
        key = tuple(sorted(int(i) for i in perms[k, :j + 1]))
        if key not in chosen:
            chosen[key] = True
            replicas += len(key)
        heap.append((-1.0, k, j))
    required = len(chosen)
    heapq.heapify(heap)
    waste = 0.0
    while heap and replicas < target_replicas:
        negp, k, j = heapq.heappop(heap)
        if j + 1 >= n:
            continue
        prev = tuple(sorted(int(i) for i in perms[k, :j + 1]))
        p = -negp * _p_continue(value(prev), mean[j + 1], sd[j + 1], v_all, truncation)
        if p <= 0.0:
            continue
        key = tuple(sorted(int(i) for i in perms[k, :j + 2]))
        if key not in chosen and value(key) is None:
            cost = (1.0 - p) * len(key)
            if waste + cost > overhead_replicas:
                continue  # not worth a batch's overhead; shallower prefixes of other walks may still be
            waste += cost
            chosen[key] = True
            replicas += len(key)
        heapq.heappush(heap, (-p, k, j + 1))
    return list(chosen), required


def wave_frontier(table, perms, v_all, truncation, interpolate, sizes, evaluate, plan=None):
    """Walk `perms` on device; while walks stop on unknown prefixes, evaluate those prefixes in one batch
    (`evaluate(list of keys) -> values`), publish them to the table and walk again.  With `plan`
    (plan(perms, stop) -> keys, e.g. plan_frontier) the batch also holds speculative deeper prefixes.
    Returns the rows."""
    while True:
        rows, status, need = tmc_walk(table, perms, v_all, truncation, interpolate, sizes)
        if np.all(status >= table.n):
            return rows
        if plan is not None:
            keys = plan(perms, status)
        else:
            keys = [mask_to_key(m) for m in sorted({int(m) for m, s in zip(need, status) if s < table.n})]
        vals = evaluate(keys)
        table.update(dict(zip(keys, (float(v) for v in vals))))


def truncated_mc_table(table, sv_accuracy=0.01, alpha=0.95, truncation=0.05, interpolate=False, sizes=None,
                       wave=100):
    """The reference TMCS / ITMCS loop (mplc/contributivity.py:215-246 / :276-316) on a fully known table:
    permutations from numpy's global RNG in the reference's order, rows computed on device in waves drawn
    ahead from a saved RNG state, stopping rule and moments in numpy.  Returns (sv, std, t)."""
    n = table.n
    v_all = float(table.V[(1 << n) - 1].item())
    q = norm.ppf((1 - alpha) / 2, loc=0, scale=1)
    contributions = np.zeros((0, n))
    t, v_max = 0, 0
    buf, pos = None, 0
    while t < 100 or t < q ** 2 * v_max / sv_accuracy ** 2:
        if buf is None or pos == len(buf[0]):
            state = np.random.get_state()
            perms = np.array([np.random.permutation(n) for _ in range(wave)])
            np.random.set_state(state)
            rows, status, _ = tmc_walk(table, perms, v_all, truncation, interpolate, sizes)
            if np.any(status < n):
                raise ValueError("truncated_mc_table needs a fully known table")
            buf, pos = (perms, rows), 0
        t += 1
        perm = np.random.permutation(n)
        assert np.array_equal(perm, buf[0][pos])
        contributions = np.vstack((contributions, buf[1][pos][None, :])) if t > 1 else buf[1][pos][None, :].copy()
        pos += 1
        v_max = np.max(np.var(contributions, axis=0))
    return np.mean(contributions, axis=0), np.std(contributions, axis=0) / np.sqrt(t - 1), t


def tmc_moments(table, n_perms, v_all=None, truncation=0.05, interpolate=False, sizes=None, perms=None, seed=0,
                perm_base=0):
    """Fixed-budget TMCS on device: (mean, std, complete) over n_perms walks (perms given or keyed on device)."""
    torch = _torch()
    n = table.n
    dev = table.device
    if v_all is None:
        v_all = float(table.V[(1 << n) - 1].item())
    lib = _native.lib()
    ws_bytes = int(lib.mplc_tmc_moments_workspace_bytes(n, int(n_perms)))
    ws = torch.empty(max(ws_bytes, 8), dtype=torch.uint8, device=dev)
    out = torch.empty(2 * n + 1, dtype=torch.float64, device=dev)
    p_d = torch.from_numpy(np.ascontiguousarray(perms, dtype=np.uint8)).to(dev) if perms is not None else None
    sz = torch.tensor(np.asarray(sizes, dtype=np.float64), device=dev) if sizes is not None else None
    _native.check(lib.mplc_tmc_moments(_native.ptr(table.V), n, _native.ptr(p_d), int(seed), int(perm_base),
                                       int(n_perms), float(v_all), float(truncation), int(bool(interpolate)),
                                       _native.ptr(sz), _native.ptr(out), _native.ptr(ws), ws_bytes,
                                       _native.stream_handle(dev)), "mplc_tmc_moments")
    m = out.cpu().numpy()
    k = m[2 * n]
    mean = m[:n] / k
    var = np.maximum(m[n:2 * n] / k - mean ** 2, 0.0)
    return mean, np.sqrt(var), int(k)


__all__ = ["VTable", "tmc_walk", "wave_frontier", "truncated_mc_table", "tmc_moments", "mask_to_key", "plan_frontier",
           "size_predictor"]
