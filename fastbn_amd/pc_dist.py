"""Multi-GPU PC-stable skeleton: one process per GPU, the column store resident on
every rank, and per level one exchange step.

The level bookkeeping is native (fastbn_amd/csrc/pc_dist.cpp, `fbn_pc_dist_*`): every rank holds
the same skeleton, cuts the level's edges into the same contiguous ranges (level 0: equal chunks of
the complete graph; level d >= 1: equal candidate-set cost C(|adj(x)|-1, d) + C(|adj(y)|-1, d) + 1),
runs its range on its own device (an edge's sequential first-independent-set search stays on one
rank) into a fixed-size int32 record, and after one all-gather of the records applies all of them
in rank order = vec_edges order, exactly as the single-GPU driver (src/PCStable.cpp:310-326).  At
level 0 the ranks also all-gather their pair tables (16 counts per pair, device to device over
RCCL) so that every rank keeps the derived level-1 counting.  This module only moves the records;
no per-edge Python.  Works with nccl (RCCL) and, for tests, with gloo (records on the CPU)."""
import ctypes as C

import numpy as np

from . import api


class PCDistSession(api._Handle):
    """One rank's view of a distributed PC-stable skeleton search (fbn_pc_dist_*)."""
    _destroy = "fbn_pc_dist_destroy"

    def __init__(self, nvars, alpha=0.05, depth=1000, group_size=1):
        h = C.c_void_p()
        api.lib.fbn_pc_dist_create(int(nvars), float(alpha), int(depth), int(group_size), C.byref(h))
        self._h, self.nvars = h, int(nvars)
        api._register(self)

    def level(self, world, rank):
        """Partition of the current level -> (d, e_begin, e_end, record_len), or None when done."""
        d, b, e, L = C.c_int(), C.c_int64(), C.c_int64(), C.c_int64()
        api.lib.fbn_pc_dist_level(self._h, int(world), int(rank), C.byref(d), C.byref(b), C.byref(e), C.byref(L))
        return None if d.value < 0 else (d.value, b.value, e.value, L.value)

    def edges(self):
        n = C.c_int64()
        api.lib.fbn_pc_dist_num_edges(self._h, C.byref(n))
        e = np.zeros((max(n.value, 1), 2), np.int32)
        api.lib.fbn_pc_dist_edges(self._h, e.ctypes.data, n.value)
        return e[:n.value]

    def run(self, ci, record_len):
        """This rank's range of the level on the device of IndependenceTest `ci` -> record."""
        rec = np.empty(record_len, np.int32)
        api.lib.fbn_pc_dist_run(self._h, ci._h, rec.ctypes.data)
        return rec

    def pack(self, removed, sepsets, counted, launched, record_len):
        """A record from results computed elsewhere (removed[n] bool, sepsets [n][d] or None)."""
        rm = np.ascontiguousarray(np.asarray(removed, np.uint8).reshape(-1))
        sp = np.ascontiguousarray(np.asarray(sepsets, np.int32)) if sepsets is not None else None
        rec = np.empty(record_len, np.int32)
        api.lib.fbn_pc_dist_pack(self._h, rm.ctypes.data if rm.size else None,
                                 sp.ctypes.data if sp is not None and sp.size else None, int(counted), int(launched),
                                 rec.ctypes.data)
        return rec

    def pairs_chunk(self):
        n = C.c_int64()
        api.lib.fbn_pc_dist_pairs_chunk(self._h, C.byref(n))
        return n.value

    def pairs_export(self, ptr, on_device):
        api.lib.fbn_pc_dist_pairs_export(self._h, C.c_void_p(ptr), int(bool(on_device)))

    def pairs_import(self, ci, ptr, on_device):
        api.lib.fbn_pc_dist_pairs_import(self._h, ci._h, C.c_void_p(ptr), int(bool(on_device)))

    def apply(self, records):
        """records [world][record_len] int32 (rank order) -> True if another level follows."""
        recs = np.ascontiguousarray(records, np.int32)
        more = C.c_int()
        api.lib.fbn_pc_dist_apply(self._h, recs.ctypes.data, C.byref(more))
        return bool(more.value)

    def result(self):
        """Skeleton + sepsets + counts + host orientation (fbn_pc_dist_result) -> api.PCResult with
        tests_per_level / launched_per_level."""
        r = C.c_void_p()
        api.lib.fbn_pc_dist_result(self._h, C.byref(r))
        return api.PCResult.with_levels(r)


def _world_rank():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def _force_exchange():
    """FBN_PC_DIST_FORCE_EXCHANGE=1: run every collective of the level loop even at world size 1
    (records and pair tables through the process group, device buffers with nccl), so a one-GPU box
    executes the RCCL data paths an 8-GPU run takes.  Testing / rehearsal switch."""
    import os
    return os.environ.get("FBN_PC_DIST_FORCE_EXCHANGE", "0") not in ("", "0")


def _all_gather_fixed(arr, device):
    """Every rank's equal-length int32 array, stacked in rank order -> numpy [world][len]."""
    import torch
    import torch.distributed as dist
    world, _ = _world_rank()
    if world == 1 and not (_force_exchange() and dist.is_available() and dist.is_initialized()):
        return arr[None, :]
    t = torch.from_numpy(arr)
    if device is not None:
        t = t.to(device)
        out = torch.empty((world, arr.size), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t)
        return out.cpu().numpy()
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return torch.stack(outs).numpy()


def _exchange_pair_tables(sess, ci, device):
    """Level 0 -> 1: all-gather every rank's chunk of pair tables into every rank's context."""
    import torch
    import torch.distributed as dist
    world, _ = _world_rank()
    chunk = sess.pairs_chunk()
    # 0: no pair tables were recorded (dataset not bit-slice eligible, or FBN_CI_NO_PAIRS).  That
    # depends on the dataset only, but the ranks agree on it explicitly before any collective that
    # assumes a chunk size: min over ranks, 0 -> every rank skips, level 1 counts without them
    if world > 1 or _force_exchange():
        chunk = int(_all_gather_fixed(np.array([chunk], np.int32), device).min())
    if chunk == 0:
        return
    on_dev = device is not None
    dev = torch.device(device) if on_dev else torch.device("cpu")
    inp = torch.zeros(chunk * 16, dtype=torch.int32, device=dev)
    sess.pairs_export(inp.data_ptr(), on_dev)
    if on_dev:
        out = torch.empty(world * chunk * 16, dtype=torch.int32, device=dev)
        dist.all_gather_into_tensor(out, inp)
        torch.cuda.synchronize(dev)
    else:
        outs = [torch.empty_like(inp) for _ in range(world)]
        dist.all_gather(outs, inp)
        out = torch.cat(outs)
    sess.pairs_import(ci, out.data_ptr(), on_dev)


def pc_skeleton_distributed(engine, nvars, alpha=0.05, depth=1000, group_size=1, device=None, ci=None):
    """Run the level loop; `engine(sess, d, b, e, record_len)` -> this rank's record for edges
    [b, e) of sess.edges() (the device engine is `sess.run(ci, record_len)`).  `device`: the torch
    device the records / pair tables travel on (an RCCL group), None for a CPU (gloo) group.  With
    `ci` given and world > 1, level 0's pair tables are all-gathered into it.  Returns the session
    after the last level (identical on every rank)."""
    world, rank = _world_rank()
    sess = PCDistSession(nvars, alpha, depth, group_size)
    while True:
        lv = sess.level(world, rank)
        if lv is None:
            break
        d, b, e, L = lv
        rec = engine(sess, d, b, e, L)
        if d == 0 and (world > 1 or _force_exchange()) and ci is not None:
            _exchange_pair_tables(sess, ci, device)
        if not sess.apply(_all_gather_fixed(rec, device)):
            break
    return sess


def pc_stable_distributed(ci, nvars, alpha=0.05, depth=1000, group_size=1, device=None):
    """Device skeleton on every rank's IndependenceTest `ci`, then host orientation ->
    (PCResult, tests_per_level, launched_per_level)."""
    sess = pc_skeleton_distributed(lambda s, d, b, e, L: s.run(ci, L), nvars, alpha, depth, group_size, device, ci)
    res = sess.result()
    return res, res.tests_per_level.tolist(), res.launched_per_level.tolist()


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
    t = broadcast_columns(cols, shape, torch.device("cuda", device), src)
    torch.cuda.synchronize(device)
    return api.IndependenceTest.from_device(t.data_ptr(), shape[0], shape[1], dims, alpha, device)


# ---------------------------------------------------------------- small graphs: replicas
# A graph the device-resident search takes (fbn_pc_small_eligible: <= 64 variables of <= 4 states,
# group size 1 -- ALARM-5000) is ONE launch of five dependent levels on one GPU (0.14 ms); cutting
# its levels over N GPUs would add an all-gather per level to that chain and cannot shorten it.
# So N GPUs run it as replicas ("replicas only"): every rank runs the whole search on
# its own copy of the broadcast column store, and ONE broadcast of rank 0's result record gives
# every rank the same answer (each rank can check its own against it).
RECORD_MAGIC = 0x52504246


def small_eligible(ci, group_size=1):
    e = C.c_int()
    api.lib.fbn_pc_small_eligible(ci._h, int(group_size), C.byref(e))
    return bool(e.value)


def record_len(handle):
    """Length (int32 words) of fbn_pc_result_record for a result handle."""
    n = C.c_int64()
    api.lib.fbn_pc_result_record(handle, None, 0, C.byref(n))
    return int(n.value)


def result_record(handle, cap=None):
    """fbn_pc_result_record of a result handle: an int32 array of exactly its length (cap=None), or
    zero-padded to `cap` (FastBNError when the record needs more)."""
    cap = record_len(handle) if cap is None else int(cap)
    rec = np.zeros(cap, np.int32)
    n = C.c_int64()
    api.lib.fbn_pc_result_record(handle, rec.ctypes.data, cap, C.byref(n))  # (raises when short)
    return rec


def unpack_record(rec):
    """-> {"tests_per_level", "edges", "sepset"} (the PCResult views) from a record."""
    r = np.asarray(rec, np.int64)
    if int(r[0]) != RECORD_MAGIC:
        raise ValueError("not a PC result record")
    L = int(r[1])
    k = 2
    tests = [int((r[k + 2 * i] & 0xFFFFFFFF) | (r[k + 2 * i + 1] << 32)) for i in range(L)]
    k += 2 * L
    ne = int(r[k])
    edges = [(int(r[k + 1 + 2 * i]), int(r[k + 2 + 2 * i])) for i in range(ne)]
    k += 1 + 2 * ne
    slen = int(r[k])
    k += 1
    sep, end = {}, k + slen
    while k < end:
        x, y, m = int(r[k]), int(r[k + 1]), int(r[k + 2])
        sep[(x, y)] = tuple(int(v) for v in r[k + 3:k + 3 + m])
        k += 3 + m
    return {"tests_per_level": tests, "edges": edges, "sepset": sep}


def broadcast_record(rec, device=None, src=0):
    """Rank `src`'s fixed-length int32 record to every rank in one broadcast (device buffers with
    nccl) -> numpy array (identity at world size 1 unless FBN_PC_DIST_FORCE_EXCHANGE)."""
    import torch
    import torch.distributed as dist
    world, _ = _world_rank()
    if world == 1 and not (_force_exchange() and dist.is_available() and dist.is_initialized()):
        return rec
    t = torch.from_numpy(np.ascontiguousarray(rec, np.int32))
    if device is not None:
        t = t.to(device)
    dist.broadcast(t, src)
    return t.cpu().numpy()


def pc_stable_replicas(ci, alpha=0.05, depth=1000, device=None, check=True):
    """Small graphs on N ranks: the whole device-resident search on every rank (fbn_pc_stable on
    its own IndependenceTest `ci`), one broadcast of rank 0's result record.  -> (PCResult of this
    rank, unpacked rank-0 record); check: every rank's own record must equal rank 0's."""
    h = C.c_void_p()
    api.lib.fbn_pc_stable(ci._h, float(alpha), int(depth), 1, C.byref(h))
    res = api.PCResult(h)
    mine = result_record(h)
    # rank 0's record length first (records are sized by the result, not by a fixed bound), then
    # the record; a rank whose own length differs still takes part in both broadcasts
    n0 = int(broadcast_record(np.array([len(mine)], np.int32), device)[0])
    buf = np.zeros(n0, np.int32)
    buf[:min(n0, len(mine))] = mine[:n0]
    got = broadcast_record(buf, device)
    if check and not (len(mine) == n0 and np.array_equal(got, mine)):
        raise RuntimeError("PC replicas disagree with rank 0's result record")
    return res, unpack_record(got)
