"""Multi-rank PC-stable on the device: fbn_pc_level ranges + one all-gather per level must give the
single-GPU driver's skeleton, sepsets, counts and orientation.  Two ranks share the one GPU of the
test box (gloo carries the exchange; on a multi-GPU node the same code runs over RCCL)."""
import os
import socket

import numpy as np
import pytest
from conftest import GOLD

import fastbn_amd as F

pytestmark = pytest.mark.gpu
CSV = os.path.join(GOLD, "alarm", "alarm_s5000.txt")
BIF = os.path.join(GOLD, "alarm", "alarm.bif")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_single_rank_level_api_matches_driver():
    from fastbn_amd import pc_dist
    ci = F.IndependenceTest(F.Dataset(CSV))
    res, tests, launched = pc_dist.pc_stable_distributed(ci, 37)
    pc = F.PCStable(0.05, 1000).StructLearnCompData(ci)
    assert res.edges == pc.edges and res.sepset == pc.sepset and tests == pc.tests_per_level.tolist()
    assert res.oriented == pc.oriented and res.GetSHD(BIF) == 5


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from fastbn_amd import pc_dist
    # rank 0 loads the file; every rank gets the column store by one broadcast (gloo carries it on
    # the CPU here; with RCCL it lands in device memory directly: independence_test_broadcast)
    ds = F.Dataset(CSV) if rank == 0 else None
    shape = [ds.num_vars, ds.num_instance] if rank == 0 else [0, 0]
    dims = ds.dims if rank == 0 else None
    meta = [shape, None if dims is None else [int(v) for v in dims]]
    dist.broadcast_object_list(meta, 0)
    t = pc_dist.broadcast_columns(ds.columns if rank == 0 else None, meta[0]).to("cuda:0")
    torch.cuda.synchronize()
    ci = F.IndependenceTest.from_device(t.data_ptr(), meta[0][0], meta[0][1], meta[1], device=0)
    res, tests, _ = pc_dist.pc_stable_distributed(ci, 37)
    if rank == 0:
        np.save(out, np.array([res.edges, sorted(res.sepset.items()), tests, res.oriented, res.GetSHD(BIF)],
                              dtype=object), allow_pickle=True)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_match_single_gpu(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "r.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    edges, sep, tests, oriented, shd = np.load(out, allow_pickle=True)  # written by this test's worker
    pc = F.PCStable(0.05, 1000).StructLearnCompData(F.Dataset(CSV))
    assert [tuple(e) for e in edges] == pc.edges
    assert dict(sep) == pc.sepset
    assert list(tests) == pc.tests_per_level.tolist()
    assert [tuple(o) for o in oriented] == pc.oriented and shd == 5


def test_from_device_matches_upload_and_rejects_bad_codes():
    import torch
    ds = F.Dataset(CSV)
    t = torch.from_numpy(np.ascontiguousarray(ds.columns)).cuda()
    ci_dev = F.IndependenceTest.from_device(t.data_ptr(), ds.num_vars, ds.num_instance, ds.dims)
    a = F.PCStable(0.05, 1000).StructLearnCompData(ci_dev)
    b = F.PCStable(0.05, 1000).StructLearnCompData(F.IndependenceTest(ds))
    assert a.edges == b.edges and a.sepset == b.sepset and a.tests_per_level.tolist() == b.tests_per_level.tolist()
    bad = ds.columns.copy()
    bad[3, 17] = ds.dims[3]  # a code outside the variable's state count
    tb = torch.from_numpy(np.ascontiguousarray(bad)).cuda()
    with pytest.raises(F.FastBNError, match="variable 3"):
        F.IndependenceTest.from_device(tb.data_ptr(), ds.num_vars, ds.num_instance, ds.dims)
    with pytest.raises(F.FastBNError, match="variable 3"):
        F.IndependenceTest(F.Dataset(columns=bad, dims=ds.dims))


def test_config5_full_size_through_session_world1():
    """BASELINE config 5 (1000 vars x 100k samples, depth 6) through the native distributed
    session at world size 1 (the N = 1 leg of bench.py's multi-GPU PC path): the fixture's
    counts, edges and sepsets, and pair tables kept for the derived level-1 counting."""
    import hashlib
    import json
    from conftest import pc_digest
    from fastbn_amd import pc_dist, synth
    ref = json.load(open(os.path.join(GOLD, "pc_c5.json")))
    cols, dims = synth.config5_dataset()
    assert hashlib.sha256(np.ascontiguousarray(cols).tobytes()).hexdigest() == ref["columns_sha256"]
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
    res, tests, launched = pc_dist.pc_stable_distributed(ci, 1000, 0.05, 6)
    assert tests == ref["tests_per_level"]
    assert pc_digest(res.edges, res.sepset) == {k: ref[k] for k in ("edges_sha256", "sepsets_sha256")}
    single = F.PCStable(0.05, 6).StructLearnCompData(ci)
    assert launched == single.launched_per_level.tolist()  # same rounds: derived level 1 kept
    assert res.oriented == single.oriented


def _worker_c5(rank, world, port, out):
    import json
    import torch.distributed as dist
    from conftest import pc_digest
    from fastbn_amd import pc_dist, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cols, dims = synth.config5_dataset()  # every rank regenerates the seeded dataset
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
    res, tests, launched = pc_dist.pc_stable_distributed(ci, 1000, 0.05, 6)
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"tests": tests, **pc_digest(res.edges, res.sepset), "oriented": len(res.oriented)}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_config5_two_ranks_vs_fixture(tmp_path):
    """BASELINE config 5 at full size on two ranks (the N > 1 path: level-0 pair ranges through the
    Gram GEMM column slices, pair tables all-gathered, device-resident level-1 search per edge range,
    one record all-gather per level; gloo carries the exchange, both ranks share the test GPU): the
    fixture's tests per level, edge list and sepsets."""
    import json
    import torch.multiprocessing as mp
    ref = json.load(open(os.path.join(GOLD, "pc_c5.json")))
    out = str(tmp_path / "c5.json")
    mp.start_processes(_worker_c5, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    got = json.load(open(out))
    assert got["tests"] == ref["tests_per_level"]
    assert {k: got[k] for k in ("edges_sha256", "sepsets_sha256")} == {k: ref[k] for k in ("edges_sha256", "sepsets_sha256")}


@pytest.mark.parametrize("knob", ["FBN_CI_NO_PAIRS", "FBN_CI_NO_BITS"])
def test_two_ranks_without_pair_tables(tmp_path, monkeypatch, knob):
    """when level 0 records no pair tables (no bit-sliced path for the dataset, or pair
    tables switched off) fbn_pc_dist_pairs_chunk reports 0 and every rank skips the exchange; level
    1 then counts without them.  Two ranks (gloo, sharing the test GPU) = the single-GPU driver."""
    import torch.multiprocessing as mp
    monkeypatch.setenv(knob, "1")  # inherited by the spawned ranks
    out = str(tmp_path / "r.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    edges, sep, tests, oriented, shd = np.load(out, allow_pickle=True)  # written by this test's worker
    pc = F.PCStable(0.05, 1000).StructLearnCompData(F.Dataset(CSV))
    assert [tuple(e) for e in edges] == pc.edges
    assert dict(sep) == pc.sepset
    assert list(tests) == pc.tests_per_level.tolist()
    assert [tuple(o) for o in oriented] == pc.oriented and shd == 5


def _worker_nccl(rank, world, port, out):
    """One rank of an RCCL ("nccl") process group on the box's GPU: configs 3 and 5 through the
    device-memory broadcast of the column store and the distributed session with every collective
    forced through the group (device all-gathers of the records and of the pair tables)."""
    import json
    import torch
    import torch.distributed as dist
    from conftest import pc_digest
    from fastbn_amd import pc_dist, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["FBN_PC_DIST_FORCE_EXCHANGE"] = "1"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    got = {}
    ds = F.Dataset(CSV)
    ci = pc_dist.independence_test_broadcast(ds.columns, [int(v) for v in ds.dims], [ds.num_vars, ds.num_instance])
    res, tests, _ = pc_dist.pc_stable_distributed(ci, 37, device="cuda:0")
    got["alarm"] = {"tests": tests, **pc_digest(res.edges, res.sepset), "shd": res.GetSHD(BIF)}
    # small graphs at N > 1: replicas + one RCCL broadcast of rank 0's result record (forced at world 1)
    rres, rec0 = pc_dist.pc_stable_replicas(ci, 0.05, 1000, device="cuda:0")
    got["alarm_replicas"] = {"tests": rec0["tests_per_level"], **pc_digest(rec0["edges"], rec0["sepset"]),
                             "shd": rres.GetSHD(BIF), "path": rres.path}
    cols, dims = synth.config5_dataset()
    ci5 = pc_dist.independence_test_broadcast(cols, [int(v) for v in dims], list(cols.shape))
    res5, tests5, _ = pc_dist.pc_stable_distributed(ci5, 1000, 0.05, 6, device="cuda:0")
    got["c5"] = {"tests": tests5, **pc_digest(res5.edges, res5.sepset)}
    if rank == 0:
        with open(out, "w") as f:
            json.dump(got, f)
    dist.barrier()
    dist.destroy_process_group()


def test_nccl_world1_forced_exchange_configs_3_and_5(tmp_path):
    """the RCCL data paths of the multi-GPU PC loop executed on one GPU -- an
    "nccl" process group of world size 1, the column store broadcast into device memory
    (independence_test_broadcast), the records and the level-0 pair tables all-gathered through
    RCCL on the device (FBN_PC_DIST_FORCE_EXCHANGE: fbn_pc_dist_pairs_export / _import with
    buf_on_device = 1).  ALARM-5000 = the single-GPU driver, config 5 = tests/golden/pc_c5.json."""
    import json
    import torch.multiprocessing as mp
    from conftest import pc_digest
    out = str(tmp_path / "nccl.json")
    mp.start_processes(_worker_nccl, args=(1, _free_port(), out), nprocs=1, join=True, start_method="spawn")
    got = json.load(open(out))
    pc = F.PCStable(0.05, 1000).StructLearnCompData(F.Dataset(CSV))
    assert got["alarm"]["tests"] == pc.tests_per_level.tolist() and got["alarm"]["shd"] == 5
    assert {k: got["alarm"][k] for k in ("edges_sha256", "sepsets_sha256")} == pc_digest(pc.edges, pc.sepset)
    rep = got["alarm_replicas"]
    assert rep["tests"] == pc.tests_per_level.tolist() and rep["shd"] == 5 and rep["path"] == 1
    assert {k: rep[k] for k in ("edges_sha256", "sepsets_sha256")} == pc_digest(pc.edges, pc.sepset)
    ref = json.load(open(os.path.join(GOLD, "pc_c5.json")))
    assert got["c5"]["tests"] == ref["tests_per_level"]
    assert {k: got["c5"][k] for k in ("edges_sha256", "sepsets_sha256")} == \
        {k: ref[k] for k in ("edges_sha256", "sepsets_sha256")}


def test_bench_gpus_2_rehearsal_on_one_gpu():
    """`bench.py --gpus 2` with no launcher starts two ranks itself (torch.distributed.run); with
    FBN_BENCH_BACKEND=gloo they share the box's GPU.  Rank 0's line: two ranks seen, the ALARM JT
    shards checked, config 5 through the distributed session equal to the fixture, and a roofline
    on every leg (the N > 1 PC legs included)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(GOLD.rstrip("/").rsplit("/", 1)[0])
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FBN_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--no-munin", "--no-loaders", "--no-baseline"], capture_output=True, text=True, env=env,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_size_seen"] == 2
    assert line["roofline"]["frac"] > 0 and line["roofline"]["full_batch_properties"]["ok"]
    assert line["pc_synthetic"]["matches_fixture"] and line["pc_synthetic"]["roofline"]["frac"] > 0
    assert line["pc_stable"]["matches_single_gpu"] and line["pc_stable"]["roofline"]["frac"] > 0


def test_bench_rccl_final_gather_at_world1():
    """The N > 1 headline's timed region over RCCL (FBN_BENCH_FORCE_GATHER=1: the process group and
    the final all-gather of every step's labels at world size 1): the line is produced and the
    gathered labels are checked inside bench.py."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(GOLD.rstrip("/").rsplit("/", 1)[0])
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["FBN_BENCH_FORCE_GATHER"] = "1"
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--steps", "3", "--warmup", "1", "--no-munin",
                        "--no-pc", "--no-loaders", "--no-baseline"], capture_output=True, text=True, env=env,
                       timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["world_size_seen"] == 1 and line["roofline"]["full_batch_properties"]["ok"]
