"""Multi-GPU plumbing for the JT path: one process per GPU, evidence cases sharded contiguously
(SURVEY §8(e)).  There is no data-path collective -- cases are independent -- only a max-over-ranks
of the timed region and, for file-driven evaluation, a gather of per-rank results.  Works with the
nccl (RCCL) backend on GPUs and with gloo on CPU (tests/test_shard.py)."""
import numpy as np


def case_shard(total, rank, world):
    """Contiguous [start, start + count) slice of `total` cases for `rank` (first ranks get +1)."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def synthetic_seed(base_seed, rank):
    """Seed of a rank's synthetic shard (bench.py: 20250131 + rank)."""
    return int(base_seed) + int(rank)


def max_over_ranks(value, device=None):
    """Max of a float over all ranks (identity without an initialized process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device=None):
    """Elementwise sum of a small float vector (MSE / HD / #correct) over all ranks."""
    import torch
    import torch.distributed as dist
    v = np.asarray(values, dtype=np.float64)
    if not (dist.is_available() and dist.is_initialized()):
        return v
    t = torch.from_numpy(v.copy()).to(device) if device is not None else torch.from_numpy(v.copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def gather_shards(local, total, device=None):
    """Concatenate every rank's contiguous shard (rows of `local`) in rank order -> [total, ...]."""
    import torch
    import torch.distributed as dist
    local = np.ascontiguousarray(local)
    if not (dist.is_available() and dist.is_initialized()):
        return local
    world = dist.get_world_size()
    counts = [case_shard(total, r, world)[1] for r in range(world)]
    cap = max(counts)
    buf = np.zeros((cap,) + local.shape[1:], dtype=local.dtype)
    buf[:local.shape[0]] = local
    t = torch.from_numpy(buf).to(device) if device is not None else torch.from_numpy(buf)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return np.concatenate([o.cpu().numpy()[:c] for o, c in zip(outs, counts)], axis=0)


def gather_var(local, device=None):
    """Concatenate variable-length row blocks of all ranks in rank order (same trailing shape)."""
    import torch
    import torch.distributed as dist
    local = np.ascontiguousarray(local)
    if not (dist.is_available() and dist.is_initialized()):
        return local
    world = dist.get_world_size()
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    counts = [int(x.item()) for x in ns]
    cap = max(max(counts), 1)
    buf = np.zeros((cap,) + local.shape[1:], dtype=local.dtype)
    buf[:local.shape[0]] = local
    t = torch.from_numpy(buf).to(device) if device is not None else torch.from_numpy(buf)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return np.concatenate([o.cpu().numpy()[:c] for o, c in zip(outs, counts)], axis=0)
