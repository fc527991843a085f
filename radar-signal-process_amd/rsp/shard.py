"""Frame sharding across GPUs: CPIs are independent, so each rank owns a
contiguous range of the CPI stream and no data crosses ranks.  The only collectives are
the timing barrier and the per-rank gathers of the elapsed time and the shard plans, all
over gloo on the host (bench.py creates no RCCL communicator: north_star's "no RCCL
collective").  In sliding-window mode (config c4) a shard also reads one
look-ahead frame (halo) owned by the next rank: see window_frames()."""


def shard_bounds(total, world, rank):
    """Contiguous [lo, hi) share of `total` units for `rank` (sizes differ by at most 1)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def weak_shard(per_rank, rank):
    """Weak scaling: every rank processes `per_rank` CPIs starting at rank * per_rank."""
    return rank * per_rank, (rank + 1) * per_rank


def window_frames(lo, hi):
    """Frames a shard of windows [lo, hi) must hold: its own plus the look-ahead frame
    (window i of frame n needs frame n+1, MTD/main_produce_dataset_win_xzr_v2.m:99,123)."""
    return lo, hi + 1


def _coll_device(dist, device):
    """gloo reduces host tensors; RCCL ("nccl") reduces device tensors."""
    return "cpu" if dist.get_backend() == "gloo" else device


def max_over_ranks(value, dist=None, device=None):
    """Max of a float over all ranks (identity without an initialised process group)."""
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=_coll_device(dist, device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(value, dist=None, device=None):
    """Every rank's float, in rank order ([value] without an initialised process group)."""
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return [float(value)]
    import torch
    dev = _coll_device(dist, device)
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]
