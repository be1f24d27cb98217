"""Multi-GPU PC-stable skeleton: one process per GPU, the column store resident on
every rank, and per level one exchange step.

Per level d the current skeleton's edges (vec_edges order) are split into contiguous ranges of
roughly equal cost -- C(|adj(x)\\{y}|, d) + C(|adj(y)\\{x}|, d) candidate sets per edge, 1 at level
0 -- each rank runs its range on its own device (`fbn_pc_level`: the edge's sequential
first-independent-set semantics stay local), and one all-gather brings every rank the removal
flags, sepsets and test counts; every rank then applies the removals in vec_edges order, exactly as
the single-GPU driver (src/PCStable.cpp:310-326).  Orientation (host) runs on the gathered skeleton.
Works with nccl (RCCL) and, for tests, with gloo."""
from math import comb

import numpy as np

from . import shard


def partition(costs, world):
    """Contiguous ranges [b, e) of near-equal total cost, one per rank (rank order)."""
    n = len(costs)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * (world - 1)
    cum = np.concatenate([[0], np.cumsum(np.asarray(costs, np.float64))])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")))
    cuts.append(n)
    cuts = [min(max(c, 0), n) for c in cuts]
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def level_costs(edges, adj, d):
    if d == 0:
        return [1.0] * len(edges)
    return [comb(len(adj[x]) - 1, d) + comb(len(adj[y]) - 1, d) + 1.0 for x, y in edges]


def pc_skeleton_distributed(level_fn, nvars, depth=1000, device=None):
    """level_fn(d, edges, b, e) -> (removed[bool], sepsets, counted, launched) for edges[b:e].
    Returns (edges, sepset dict, tests_per_level, launched_per_level), identical on every rank."""
    import torch.distributed as dist
    world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
    rank = dist.get_rank() if world > 1 else 0
    edges = [(i, j) for i in range(nvars) for j in range(i + 1, nvars)]
    adj = [[j for j in range(nvars) if j != i] for i in range(nvars)]
    sepset, tests, launched = {}, [], []
    d = 0
    while d == 0 or d < depth:
        ranges = partition(level_costs(edges, adj, d), world)
        b, e = ranges[rank]
        rm, seps, cnt, lau = level_fn(d, edges, b, e)
        # one exchange: removal flags + sepsets (fixed width d, -1 = kept) + counts, rank order
        width = max(d, 1)
        rec = np.full((e - b, 1 + width), -1, np.int32)
        rec[:, 0] = np.asarray(rm, np.int32)
        for i, z in enumerate(seps):
            if z is not None and d:
                rec[i, 1:1 + d] = z
        allrec = shard.gather_var(rec, device)
        cnts = shard.sum_over_ranks([cnt, lau], device)
        assert allrec.shape[0] == len(edges)
        keep = []
        for (x, y), r in zip(edges, allrec):
            if r[0]:
                sepset[(x, y)] = tuple(int(v) for v in r[1:1 + d]) if d else ()
            else:
                keep.append((x, y))
        edges = keep
        adj = [[] for _ in range(nvars)]
        for x, y in edges:
            adj[x].append(y)
            adj[y].append(x)
        tests.append(int(cnts[0]))
        launched.append(int(cnts[1]))
        if d >= 1 and not (max(len(a) for a in adj) - 1 > d):
            break
        d += 1
    return edges, sepset, tests, launched


def broadcast_columns(cols, shape, device=None, src=0):
    """The read-only column store from rank `src` to every rank in one broadcast:
    `cols` = uint8 [nvars][nsamples] numpy array on `src` (ignored elsewhere), `shape` = (nvars,
    nsamples) on every rank.  Returns a uint8 torch tensor on `device` (CPU for gloo) holding the
    columns on every rank; with nccl (RCCL) it stays on the GPU for IndependenceTest.from_device."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cpu") if device is None else torch.device(device)
    if dist.get_rank() == src:
        t = torch.from_numpy(np.ascontiguousarray(cols, np.uint8)).to(dev)
    else:
        t = torch.empty(tuple(shape), dtype=torch.uint8, device=dev)
    dist.broadcast(t, src)
    return t


def independence_test_broadcast(cols, dims, shape, alpha=0.05, device=0, src=0):
    """Every rank's IndependenceTest over the column store loaded on rank `src`, moved by one RCCL
    broadcast straight into device memory (no host copy on the receiving ranks)."""
    import torch
    from . import api
    t = broadcast_columns(cols, shape, torch.device("cuda", device), src)
    torch.cuda.synchronize(device)
    return api.IndependenceTest.from_device(t.data_ptr(), shape[0], shape[1], dims, alpha, device)


def pc_stable_distributed(ci, nvars, alpha=0.05, depth=1000, group_size=1, device=None):
    """Device skeleton on every rank's IndependenceTest `ci`, then host orientation."""
    from . import api

    def level_fn(d, edges, b, e):
        return ci.level(d, edges, b, e, group_size)

    edges, sepset, tests, launched = pc_skeleton_distributed(level_fn, nvars, depth, device)
    return api.orient_skeleton(nvars, edges, sepset), tests, launched
