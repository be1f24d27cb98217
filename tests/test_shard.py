"""N>1 path of the JT bench / evaluation on CPU: world_size-2 gloo process group, each rank computes
its contiguous shard (here with the CPU oracle standing in for the GPU kernel), results gathered and
compared with a single-process run; max-over-ranks timing reduction."""
import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

from fastbn_amd import shard  # noqa: E402


def test_case_shard_partition():
    for total in (0, 1, 63, 100000, 100003):
        for world in (1, 2, 3, 8):
            parts = [shard.case_shard(total, r, world) for r in range(world)]
            assert sum(c for _, c in parts) == total
            assert parts[0][0] == 0
            for (s0, c0), (s1, _) in zip(parts, parts[1:]):
                assert s0 + c0 == s1
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, xml, ev_path, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    ev = np.load(ev_path)
    start, count = shard.case_shard(ev.shape[0], rank, world)
    lab, marg = O.OracleJT(xml).infer(ev[start:start + count])
    labels = shard.gather_shards(lab, ev.shape[0])
    margs = shard.gather_shards(marg, ev.shape[0])
    tmax = shard.max_over_ranks(float(rank + 1))
    sums = shard.sum_over_ranks([float(count), float((lab == 0).sum())])
    if rank == 0:
        np.savez(out_path, labels=labels, margs=margs, tmax=tmax, sums=sums)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_match_single_process(tmp_path):
    mp = pytest.importorskip("torch.multiprocessing")
    import oracle as O
    from fastbn_amd import synth
    xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
    ev = synth.evidence_cases(synth.read_xmlbif(xml), 301, 7, seed=shard.synthetic_seed(20250131, 0))
    ev_path = str(tmp_path / "ev.npy")
    np.save(ev_path, ev)
    out = str(tmp_path / "out.npz")
    mp.start_processes(_worker, args=(2, _free_port(), xml, ev_path, out), nprocs=2, join=True,
                       start_method="spawn")
    r = np.load(out)
    lab, marg = O.OracleJT(xml).infer(ev)
    np.testing.assert_array_equal(r["labels"], lab)
    np.testing.assert_array_equal(r["margs"], marg)
    assert float(r["tmax"]) == 2.0
    assert r["sums"][0] == 301 and r["sums"][1] == (lab == 0).sum()


# ---------------------------------------------------------------- multi-GPU PC-stable orchestration
def _oracle_level_fn(od):
    """Per-edge CheckEdge restated over the oracle's CI test (group size 1): the CPU stand-in for
    fbn_pc_level in the orchestration tests."""
    from itertools import combinations

    def level_fn(d, edges, b, e):
        adj = {}
        for x, y in edges:
            adj.setdefault(x, []).append(y)
            adj.setdefault(y, []).append(x)
        rm, seps, cnt = [], [], 0
        for x, y in edges[b:e]:
            if d == 0:
                cnt += 1
                ind = od.ci_test(x, y)["is_independent"]
                rm.append(ind)
                seps.append(() if ind else None)
                continue
            found = None
            for a, other in ((x, y), (y, x)):
                cand = sorted(v for v in adj[a] if v != other)
                for z in combinations(cand, d):
                    cnt += 1
                    if od.ci_test(x, y, list(z))["is_independent"]:
                        found = tuple(sorted(z))
                        break
                if found is not None:
                    break
            rm.append(found is not None)
            seps.append(found)
        return rm, seps, cnt, cnt
    return level_fn


def _oracle_engine(od):
    """The session's engine on the CPU: the oracle restatement of CheckEdge over the range."""
    def engine(sess, d, b, e, L):
        edges = [tuple(map(int, x)) for x in sess.edges()]
        rm, seps, cnt, lau = _oracle_level_fn(od)(d, edges, b, e)
        sp = np.full((len(rm), max(d, 1)), -1, np.int32)
        for i, z in enumerate(seps):
            if z is not None and d:
                sp[i, :d] = z
        return sess.pack(np.asarray(rm, np.uint8), sp if d else None, cnt, lau, L)
    return engine


def _pc_worker(rank, world, port, csv, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from fastbn_amd import pc_dist
    od = O.OracleDataset(csv=csv)
    sess = pc_dist.pc_skeleton_distributed(_oracle_engine(od), 37)
    res = sess.result()
    if rank == 0:
        np.save(out_path, np.array([res.edges, sorted(res.sepset.items()), res.tests_per_level.tolist(),
                                    res.oriented], dtype=object), allow_pickle=True)
    dist.barrier()
    dist.destroy_process_group()


def test_session_partition_is_deterministic_and_balanced():
    """fbn_pc_dist_level on W independent sessions (one per simulated rank): the same contiguous
    cover of the level's edges on every rank; level 0 in equal chunks of the complete graph; after
    applying the same records, level 1 cut by candidate-set cost."""
    from fastbn_amd import pc_dist
    n = 70  # 2415 pairs: ranges start off the 32-pair record words
    for world in (1, 2, 3, 8):
        ss = [pc_dist.PCDistSession(n, 0.05, 3) for _ in range(world)]
        lv = [s.level(world, r) for r, s in enumerate(ss)]
        P = n * (n - 1) // 2
        chunk = -(-P // world)
        assert [x[1] for x in lv] == [min(P, r * chunk) for r in range(world)]
        assert lv[-1][2] == P and all(a[2] == b[1] for a, b in zip(lv, lv[1:]))
        assert len({x[3] for x in lv}) == 1  # same record length everywhere
        rng = np.random.default_rng(world)
        rm_all = rng.random(P) < 0.7  # drop ~70 % of the pairs at level 0
        # removal flags are "nonzero = removed" at the C-ABI: any byte value packs to one bit
        flags = np.where(rm_all, rng.integers(1, 256, P), 0).astype(np.uint8)
        recs = np.stack([s.pack(flags[b:e], None, e - b, e - b, L) for s, (_, b, e, L) in zip(ss, lv)])
        for s in ss:
            assert s.apply(recs)
        lv1 = [s.level(world, r) for r, s in enumerate(ss)]
        E = len(ss[0].edges())
        assert E == int((~rm_all).sum())
        iu = np.triu_indices(n, 1)  # pair order of the complete graph
        np.testing.assert_array_equal(ss[0].edges(), np.stack(iu, 1)[~rm_all])
        assert lv1[0][1] == 0 and lv1[-1][2] == E and all(a[2] == b[1] for a, b in zip(lv1, lv1[1:]))
        assert all(np.array_equal(ss[0].edges(), s.edges()) for s in ss)
        assert len({x[1:] for x in lv1}) == world or E < world
        # balance: candidate-set cost per range within one edge's cost of the ideal share
        edges = ss[0].edges()
        deg = np.bincount(edges.reshape(-1), minlength=n)
        cost = (deg[edges[:, 0]] - 1).clip(0) + (deg[edges[:, 1]] - 1).clip(0) + 1.0
        share = cost.sum() / world
        for _, b, e, _ in lv1:
            assert abs(cost[b:e].sum() - share) <= cost.max() + 1e-9


def test_session_single_rank_matches_oracle():
    """world_size 1 through the session with the oracle as the engine: the restatement's skeleton."""
    import oracle as O
    from fastbn_amd import pc_dist
    csv = os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt")
    od = O.OracleDataset(csv=csv)
    res = pc_dist.pc_skeleton_distributed(_oracle_engine(od), 37).result()
    ref = od.pc_stable(0.05, 1000, 1)
    assert res.edges == [tuple(e) for e in ref["edges"]]
    assert res.sepset == {k: tuple(v) for k, v in ref["sepset"].items()}
    assert res.tests_per_level.tolist() == list(ref["tests_per_level"])


def test_two_rank_gloo_pc_skeleton_matches_oracle(tmp_path):
    """world_size 2: per-level edge partition + one all-gather == the single-process reference order."""
    mp = pytest.importorskip("torch.multiprocessing")
    import oracle as O
    csv = os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt")
    out = str(tmp_path / "pc.npy")
    mp.start_processes(_pc_worker, args=(2, _free_port(), csv, out), nprocs=2, join=True, start_method="spawn")
    edges, sep, tests, oriented = np.load(out, allow_pickle=True)  # written by this test's own worker
    ref = O.OracleDataset(csv=csv).pc_stable(0.05, 1000, 1)
    ref_sep = {k: tuple(v) for k, v in ref["sepset"].items()}
    assert [tuple(e) for e in edges] == [tuple(e) for e in ref["edges"]]
    assert dict(sep) == ref_sep
    assert list(tests) == list(ref["tests_per_level"])
    import orient
    assert [tuple(o) for o in oriented] == orient.orient(37, [tuple(e) for e in ref["edges"]], ref_sep)


def _bcast_worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastbn_amd import pc_dist
    cols = np.random.default_rng(7).integers(0, 4, (37, 5000)).astype(np.uint8) if rank == 0 else None
    t = pc_dist.broadcast_columns(cols, (37, 5000))
    np.save(f"{out_path}.{rank}.npy", t.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_column_broadcast(tmp_path):
    """The column store loaded on rank 0 reaches every rank by one broadcast."""
    mp = pytest.importorskip("torch.multiprocessing")
    out = str(tmp_path / "cols")
    mp.start_processes(_bcast_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    ref = np.random.default_rng(7).integers(0, 4, (37, 5000)).astype(np.uint8)
    for r in range(2):
        np.testing.assert_array_equal(np.load(f"{out}.{r}.npy"), ref)


# ---------------------------------------------------------------- small graphs: replicas
def _replica_worker(rank, world, port, csv, out_path):
    """Every rank computes the whole skeleton itself (the oracle stands in for the one-launch device
    search), packs it with the native fbn_pc_result_record, and rank 0's record is broadcast."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    import fastbn_amd as F
    from fastbn_amd import pc_dist
    ref = O.OracleDataset(csv=csv).pc_stable(0.05, 1000, 1)
    res = F.orient_skeleton(37, ref["edges"], {tuple(k): tuple(v) for k, v in ref["sepset"].items()})
    mine = pc_dist.result_record(res._h)
    got = pc_dist.broadcast_record(mine)
    out = pc_dist.unpack_record(got)
    np.save(f"{out_path}.{rank}.npy", np.array([out["edges"], sorted(out["sepset"].items()),
                                                bool(np.array_equal(got, mine))], dtype=object), allow_pickle=True)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_pc_replicas_record(tmp_path):
    """Small graphs at N > 1 (bench.py / CLI): replicas + one broadcast of rank 0's result record;
    every rank decodes the single-process skeleton and sepsets and agrees with its own record."""
    mp = pytest.importorskip("torch.multiprocessing")
    import oracle as O
    csv = os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt")
    out = str(tmp_path / "rep")
    mp.start_processes(_replica_worker, args=(2, _free_port(), csv, out), nprocs=2, join=True,
                       start_method="spawn")
    ref = O.OracleDataset(csv=csv).pc_stable(0.05, 1000, 1)
    for r in range(2):
        edges, sep, same = np.load(f"{out}.{r}.npy", allow_pickle=True)  # written by this test's own workers
        assert [tuple(e) for e in edges] == [tuple(e) for e in ref["edges"]]
        assert dict(sep) == {k: tuple(v) for k, v in ref["sepset"].items()}
        assert same
