"""Multi-GPU coalition sharding (one process per GPU, torch.distributed over RCCL/xGMI).

The reference is single-process.  Coalition trainings are independent, so the
only exchanges are:
  - v(S) assembly: every rank trains an LPT share of the requested coalitions (cost ~ sum of partner
    sizes, so ranks get equal replica-steps) and the values are combined with ONE all_reduce(sum) of a
    dense fp64 vector (each coalition is owned by exactly one rank, others contribute 0);
  - range-sharded exact Shapley (n >= 16): each rank reduces its mask range, partial sums all_reduced
    (mplc.shapley.ShapleyAggregator.partial / finalize).
With early stopping a coalition's cost is its rows times its REALISED epochs, which vary (15-28 of 40 for config #3
at the reference's defaults).  EpochModel learns the realised epochs per coalition size from the batches already
trained - carried in the same all_reduce as the values, so every rank holds the same model and computes the same
plan - and scales the LPT cost by the predicted epochs.  v(S) depends only on (S, seed), so the
plan never changes a value.
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


def coalition_cost(coalition, partner_sizes, epochs=1.0):
    """LPT cost of training a coalition: its partners' rows (replica-steps per epoch) times the epochs it trains."""
    return float(sum(partner_sizes[p] for p in coalition)) * float(epochs)


class EpochModel:
    """Realised training epochs per coalition size (early stopping), learned from the coalitions already trained:
    predict(k) = the mean over size k once MIN_SEEN of that size are known, else the mean over all sizes, else the
    configured epoch count.  Updated only with all-reduced data, so identical on every rank."""
    MIN_SEEN = 4

    def __init__(self, epochs):
        self.epochs = float(epochs)
        self.sum, self.cnt = {}, {}

    def update(self, coalitions, epochs_done):
        for c, e in zip(coalitions, epochs_done):
            k = len(c)
            self.sum[k] = self.sum.get(k, 0.0) + float(e)
            self.cnt[k] = self.cnt.get(k, 0) + 1

    def predict(self, k):
        if self.cnt.get(k, 0) >= self.MIN_SEEN:
            return self.sum[k] / self.cnt[k]
        n = sum(self.cnt.values())
        return sum(self.sum.values()) / n if n else self.epochs


def sharded_evaluate(evaluate_local, coalitions, partner_sizes, device=None, epochs_local=None, epoch_model=None):
    """Evaluate `coalitions` across all ranks; every rank returns the full float64 value vector.
    epochs_local() (optional) returns the realised epochs of the coalitions the last evaluate_local call trained;
    with an `epoch_model` (EpochModel) they weight the LPT costs and the model is updated with every rank's epochs,
    which travel in the values' all_reduce."""
    import torch
    import torch.distributed as dist
    rank, ws = world()
    C = len(coalitions)
    track = epochs_local is not None and epoch_model is not None
    if ws == 1:
        vals = np.asarray(evaluate_local(coalitions), dtype=np.float64)
        if track:
            epoch_model.update(coalitions, epochs_local())
        return vals
    w = (lambda c: epoch_model.predict(len(c))) if epoch_model is not None else (lambda c: 1.0)
    shards = lpt_shard([coalition_cost(c, partner_sizes, w(c)) for c in coalitions], ws)
    mine = shards[rank]
    buf = np.zeros(2 * C if track else C, dtype=np.float64)  # [values | realised epochs]
    if mine:
        buf[mine] = evaluate_local([coalitions[i] for i in mine])
        if track:
            buf[C + np.asarray(mine)] = np.asarray(epochs_local(), dtype=np.float64)
    backend = dist.get_backend()
    dev = device if (backend == "nccl" and device is not None) else torch.device("cpu")
    t = torch.from_numpy(buf).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    out = t.cpu().numpy()
    if track:
        epoch_model.update(coalitions, out[C:])
    return out[:C]


__all__ = ["lpt_shard", "sharded_evaluate", "world", "coalition_cost", "EpochModel"]
