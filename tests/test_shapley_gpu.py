"""GPU parity: the HIP exact-Shapley kernel vs the reference outputs and the long-double oracle.

Tolerance (north star): 1e-12 relative to the reference fp64 computation."""
import json
import os

import numpy as np
import pytest

from oracle import shapley as osh

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "shapley_value.json")
RTOL = 1e-12


def _rel(a, b):
    return np.max(np.abs(np.asarray(a) - np.asarray(b))) / np.max(np.abs(b))


def test_drop_in_shapley_value_vs_reference_goldens():
    from mplc.shapley import shapley_value
    with open(GOLDEN) as f:
        cases = json.load(f)["data"]
    for c in cases:
        out = shapley_value(c["n"], c["v_combination_order"])
        assert len(out) == c["n"]
        assert _rel(out, c["shapley"]) <= RTOL, c["n"]


@pytest.mark.parametrize("n", [1, 3, 9, 15, 16, 17, 20, 24])
def test_bitmask_kernel_vs_long_double_oracle(n):
    from mplc.shapley import shapley_from_table
    V = osh.synthetic_table(n, seed_s=n, seed_u=n + 1)
    ref = osh.shapley_bitmask_ld(n, V)
    out = shapley_from_table(V, n)
    assert _rel(out, ref) <= RTOL


def test_ragged_values_and_negative_entries():
    from mplc.shapley import shapley_from_table
    n = 18
    V = np.random.default_rng(3).normal(size=1 << n)
    V[0] = 0.0
    ref = osh.shapley_bitmask_ld(n, V)
    assert _rel(shapley_from_table(V, n), ref) <= 1e-11


def test_range_sharded_partials_sum_to_exact():
    import torch
    from mplc.shapley import ShapleyAggregator, shard_range
    n = 20
    V = torch.from_numpy(osh.synthetic_table(n)).cuda()
    agg = ShapleyAggregator(n)
    exact = agg.run(V).clone()
    for world in (2, 4, 8):
        tot = torch.zeros(2 * (n + 1), dtype=torch.float64, device="cuda")
        for r in range(world):
            b, e = shard_range(n, r, world)
            tot += agg.partial(V[b:e], b)
        sv = agg.finalize(tot)
        assert _rel(sv.cpu().numpy(), exact.cpu().numpy()) <= 1e-13


def test_n28_properties():
    """Full-size table (2^28 fp64 = 2 GiB): efficiency (sum SV = v(N)), symmetry, and linearity."""
    import torch
    from mplc.shapley import ShapleyAggregator
    n = 28
    idx = torch.arange(1 << n, device="cuda", dtype=torch.int64)
    pc = torch.zeros_like(idx)
    for i in range(n):
        pc += (idx >> i) & 1
    # symmetric game v(S) = f(|S|): all SV equal to f(n)/n
    V = (1.0 - torch.exp(-pc.double() / 7.0))
    V[0] = 0.0
    agg = ShapleyAggregator(n)
    sv = agg.run(V).cpu().numpy()
    assert np.max(np.abs(sv - V[-1].item() / n)) <= RTOL * abs(V[-1].item() / n)
    # additive game v(S) = sum_{i in S} c_i: SV_i = c_i exactly (linearity + dummy)
    c = torch.linspace(0.1, 2.8, n, dtype=torch.float64, device="cuda")
    V2 = torch.zeros(1 << n, dtype=torch.float64, device="cuda")
    for i in range(n):
        V2 += ((idx >> i) & 1).double() * c[i]
    sv2 = agg.run(V2).cpu().numpy()
    assert _rel(sv2, c.cpu().numpy()) <= RTOL
    # linearity: SV(V + V2) = SV(V) + SV(V2)
    V3 = V + V2
    sv3 = agg.run(V3).cpu().numpy()
    assert _rel(sv3, sv + sv2) <= RTOL
    # efficiency on a generic table
    V4 = V * (1.0 + 0.01 * torch.sin(idx.double()))
    V4[0] = 0
    sv4 = agg.run(V4).cpu().numpy()
    assert abs(sv4.sum() - V4[-1].item()) <= 1e-12


def test_fedavg_aggregate_bit_exact_vs_np_average():
    """mplc_fedavg_aggregate == np.average(axis=0, weights=w) of mplc/mpl_utils.py:96-100, cast to fp32."""
    import torch
    from mplc.fedavg import fedavg_aggregate, aggregation_weights
    rng = np.random.default_rng(0)
    sizes_list = [[437, 3936], [874, 2186, 1312], [4374] * 9 + [4373], [57, 56, 57]]
    n_param = 1199882
    for sizes in sizes_list:
        P = len(sizes)
        x = rng.normal(scale=0.05, size=(P, n_param)).astype(np.float32)
        for scheme in ("data-volume", "uniform"):
            w, scl = aggregation_weights(sizes, scheme)
            ref = np.average(x.astype(np.float32), axis=0, weights=np.asarray(w)).astype(np.float32)
            xt = torch.from_numpy(x).cuda()
            out = fedavg_aggregate([xt], [list(range(P))], [sizes], scheme=scheme)[0].cpu().numpy()
            assert np.array_equal(out, ref), (sizes, scheme)


def test_fedavg_bcast_skip_leaves_range_in_the_replicas():
    """mplc_fedavg_aggregate_bcast_skip: the average in the coalition row, written back into every replica row
    except [skip_lo, skip_hi) (the MNIST W3, which the next round's first step reads from the coalition row)."""
    import torch
    from mplc import _native
    from mplc.fedavg import aggregation_weights
    rng = np.random.default_rng(1)
    sizes = [874, 2186, 1312]
    P, n_param, stride = 3, 1199882, 1199936
    x = np.zeros((P, stride), dtype=np.float32)
    x[:, :n_param] = rng.normal(scale=0.05, size=(P, n_param))
    w, scl = aggregation_weights(sizes, "data-volume")
    ref = np.average(x[:, :n_param], axis=0, weights=np.asarray(w)).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    out = torch.zeros((1, stride), dtype=torch.float32, device="cuda")
    first = torch.tensor([0, P], dtype=torch.int32, device="cuda")
    wt = torch.tensor(w, dtype=torch.float64, device="cuda")
    st = torch.tensor([scl], dtype=torch.float64, device="cuda")
    lo, hi = 18816, 1198464
    _native.check(_native.lib().mplc_fedavg_aggregate_bcast_skip(
        _native.ptr(xt), stride, _native.ptr(first), _native.ptr(wt), _native.ptr(st), 1, n_param,
        _native.ptr(out), stride, lo, hi, _native.stream_handle()), "mplc_fedavg_aggregate_bcast_skip")
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy()[0, :n_param], ref)
    after = xt.cpu().numpy()
    for r in range(P):
        assert np.array_equal(after[r, :lo], ref[:lo]) and np.array_equal(after[r, hi:n_param], ref[hi:])
        assert np.array_equal(after[r, lo:hi], x[r, lo:hi])
    # without an output row the skipped range would be lost: refused
    assert _native.lib().mplc_fedavg_aggregate_bcast_skip(
        _native.ptr(xt), stride, _native.ptr(first), _native.ptr(wt), _native.ptr(st), 1, n_param,
        None, stride, lo, hi, _native.stream_handle()) != 0
