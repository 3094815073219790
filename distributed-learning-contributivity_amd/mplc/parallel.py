"""Multi-GPU coalition sharding (one process per GPU, torch.distributed over RCCL/xGMI).

The reference is single-process.  Coalition trainings are independent, so the
only exchanges are:
  - v(S) assembly: every rank trains an LPT share of the requested coalitions (cost ~ sum of partner
    sizes, so ranks get equal replica-steps) and the values are combined with ONE all_reduce(sum) of a
    dense fp64 vector (each coalition is owned by exactly one rank, others contribute 0);
  - range-sharded exact Shapley (n >= 16): each rank reduces its mask range, partial sums all_reduced
    (mplc.shapley.ShapleyAggregator.partial / finalize).
No communication happens during training.  Works with the gloo backend on CPU for the host logic
(tests/test_parallel.py) and with nccl (= RCCL) on the MI355X.
"""
import numpy as np


def world():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except Exception:
        pass
    return 0, 1


def lpt_shard(costs, world_size):
    """Longest-processing-time-first assignment: list of index lists, one per rank, balanced by cost.
    Deterministic (ties broken by index) so every rank computes the same plan without communication."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    loads = [0.0] * world_size
    shards = [[] for _ in range(world_size)]
    for i in order:
        r = min(range(world_size), key=lambda k: (loads[k], k))
        shards[r].append(i)
        loads[r] += costs[i]
    return [sorted(s) for s in shards]


def coalition_cost(coalition, partner_sizes):
    return float(sum(partner_sizes[p] for p in coalition))


def sharded_evaluate(evaluate_local, coalitions, partner_sizes, device=None):
    """Evaluate `coalitions` across all ranks; every rank returns the full float64 value vector."""
    import torch
    import torch.distributed as dist
    rank, ws = world()
    if ws == 1:
        return np.asarray(evaluate_local(coalitions), dtype=np.float64)
    shards = lpt_shard([coalition_cost(c, partner_sizes) for c in coalitions], ws)
    mine = shards[rank]
    vals = np.zeros(len(coalitions), dtype=np.float64)
    if mine:
        vals[mine] = evaluate_local([coalitions[i] for i in mine])
    backend = dist.get_backend()
    dev = device if (backend == "nccl" and device is not None) else torch.device("cpu")
    t = torch.from_numpy(vals).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


__all__ = ["lpt_shard", "sharded_evaluate", "world", "coalition_cost"]
