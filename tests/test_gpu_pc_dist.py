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
    from fastbn_amd import pc_dist
    ci = F.IndependenceTest(F.Dataset(CSV), device=0)
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
