"""GPU, two processes (gloo rendezvous, both ranks on cuda:0 of the 1-GPU box): the product multi-rank path.
- compute_SV at n = 16 partners: v(S) LPT-sharded through mplc.parallel.sharded_evaluate (a fixed v(S)
  table stands in for training), then the exact Shapley sum range-sharded by mplc.shapley.sharded_shapley:
  each rank reduces half of the 2^16 masks on the HIP kernel, the partials are all_reduced.  Both ranks
  must hold the single-process result (1e-12 relative) and the same memo / call count.
- shapley_from_table at n = 20 against the long-double oracle.
The 8-GPU runs use the same code with nccl (RCCL)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _table(n):
    """v(S) of the coalitions (sorted tuples) - a smooth saturating game with a little noise."""
    from itertools import combinations
    rng = np.random.default_rng(5)
    s = rng.uniform(1.0, 3.0, size=n)
    noise = rng.uniform(-1e-3, 1e-3, size=1 << n)
    out = {}
    for r in range(1, n + 1):
        for c in combinations(range(n), r):
            m = sum(1 << i for i in c)
            out[c] = 1.0 - np.exp(-s[list(c)].sum() / (s.sum() / 4)) + noise[m]
    return s, out


def _compute_sv(n, table):
    import types
    from mplc.contributivity import Contributivity
    from mplc.parallel import sharded_evaluate
    sizes = [100 + i for i in range(n)]

    class Approach:
        @staticmethod
        def evaluate_coalitions(scenario, cs):
            return sharded_evaluate(lambda cc: np.array([table[c] for c in cc]), list(cs), sizes)

    partners = [types.SimpleNamespace(id=i, y_train=np.zeros(sz)) for i, sz in enumerate(sizes)]
    sc = types.SimpleNamespace(partners_list=partners, multi_partner_learning_approach=Approach)
    c = Contributivity(scenario=sc)
    c.compute_contributivity("Shapley values")
    return c


def _worker(rank, world, port, out_q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "distributed-learning-contributivity_amd"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import shapley as osh
    from mplc.shapley import shapley_from_table
    n = 16
    _, table = _table(n)
    c = _compute_sv(n, table)
    V = osh.synthetic_table(20)
    sv20 = shapley_from_table(V, 20, sharded=True)
    sv20_local = shapley_from_table(V, 20)  # default: local, no collective
    out_q.put((rank, c.contributivity_scores.tolist(), c.first_charac_fct_calls_count, sv20.tolist(),
               sv20_local.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_compute_sv_range_sharded():
    import torch.multiprocessing as mp
    from oracle import shapley as osh
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1:] == res[1][1:]  # both ranks hold the same result
    n = 16
    _, table = _table(n)
    single = _compute_sv(n, table)  # this process: world size 1, one-pass kernel
    sv = np.array(res[0][1])
    assert np.max(np.abs(sv - single.contributivity_scores)) <= 1e-12 * np.max(np.abs(single.contributivity_scores))
    assert res[0][2] == single.first_charac_fct_calls_count == 2 ** n - 1
    ref20 = osh.shapley_bitmask_ld(20, osh.synthetic_table(20))
    assert np.max(np.abs(np.array(res[0][3]) - ref20)) <= 1e-12 * np.max(np.abs(ref20))
    assert np.max(np.abs(np.array(res[0][4]) - ref20)) <= 1e-12 * np.max(np.abs(ref20))
