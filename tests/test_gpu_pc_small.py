"""The device-resident PC-stable skeleton search for small graphs (fastbn_amd/csrc/pc_small.hip: one
launch runs every level, one grid barrier per level) against the restatement (oracle/pc_oracle.cpp)
and against the host-driven level loop (FBN_PC_NO_SMALL): tests per level, skeleton (vec_edges
order), sepsets, orientation.  launched: levels 1-2 evaluate every edge's first 8 candidate sets, then
skip the rest of an edge once an independent set at a lower index is published (timing-dependent,
between the counted tests and full speculation); levels 0, 3, 4 evaluate every candidate set."""
import os

import numpy as np
import pytest
from conftest import GOLD

import fastbn_amd as F
import oracle as O

pytestmark = pytest.mark.gpu
CSV = os.path.join(GOLD, "alarm", "alarm_s5000.txt")


def _host(ds, alpha, depth, monkeypatch):
    monkeypatch.setenv("FBN_PC_NO_SMALL", "1")
    try:
        return F.PCStable(alpha, depth).StructLearnCompData(ds)
    finally:
        monkeypatch.delenv("FBN_PC_NO_SMALL")


def _check(ds, od, alpha, depth, monkeypatch, host=True):
    ref = od.pc_stable(alpha, depth, 1)
    pc = F.PCStable(alpha, depth).StructLearnCompData(ds)
    assert pc.tests_per_level.tolist() == ref["tests_per_level"]
    assert pc.edges == ref["edges"]
    assert pc.sepset == ref["sepset"]
    if host:
        h = _host(ds, alpha, depth, monkeypatch)
        assert pc.tests_per_level.tolist() == h.tests_per_level.tolist()
        assert pc.edges == h.edges and pc.sepset == h.sepset and pc.oriented == h.oriented
    return pc


@pytest.fixture(scope="module")
def alarm():
    return F.Dataset(CSV), O.OracleDataset(csv=CSV)


def test_alarm5000_default_is_device_resident(alarm, monkeypatch):
    ds, od = alarm
    pc = _check(ds, od, 0.05, 1000, monkeypatch)
    assert pc.tests_per_level.tolist() == [666, 3579, 828, 118, 15] and len(pc.edges) == 44
    # levels 0, 3, 4: every candidate set once; 1, 2: full speculation minus the part-B skips; level 1
    # also minus the candidates the information screen decides (certainly dependent: not run)
    la = pc.launched_per_level.tolist()
    assert la[0] == 666 and la[3:] == [128, 15]
    assert 0 < la[1] < 3579 and 828 <= la[2] <= 1212
    monkeypatch.setenv("FBN_PC_NO_MISCREEN", "1")  # the screen off: the same answer, every candidate run
    ns = F.PCStable(0.05, 1000).StructLearnCompData(F.IndependenceTest(ds))
    monkeypatch.delenv("FBN_PC_NO_MISCREEN")
    assert ns.tests_per_level.tolist() == pc.tests_per_level.tolist()
    assert ns.edges == pc.edges and ns.sepset == pc.sepset and ns.oriented == pc.oriented
    assert 3579 <= ns.launched_per_level.tolist()[1] <= 8732
    assert pc.GetSHD(os.path.join(GOLD, "alarm", "alarm.bif")) == 5
    assert pc.near_alpha == 0 and pc.min_margin > 1e-9


@pytest.mark.parametrize("alpha,depth", [(0.0, 1000), (0.001, 1000), (0.01, 1000), (0.2, 1000), (0.5, 1000),
                                         (1.0, 3)])
def test_alarm5000_alphas(alarm, alpha, depth, monkeypatch):
    """alpha 1: nothing but df-0 tests is independent, the graph stays (nearly) complete -- depth 3
    keeps the restatement's CPU run short."""
    ds, od = alarm
    _check(ds, od, alpha, depth, monkeypatch)


@pytest.mark.parametrize("depth", [1, 2, 3, 4])
def test_alarm5000_depths(alarm, depth, monkeypatch):
    ds, od = alarm
    pc = _check(ds, od, 0.05, depth, monkeypatch)
    assert len(pc.tests_per_level) == depth


@pytest.mark.parametrize("ns,nv", [(1, 6), (33, 12), (4999, 40), (20011, 64)])
def test_synthetic_ragged_sizes(tmp_path, ns, nv, monkeypatch):
    """Ragged sample counts (bit-sliced tail words, 2-bit packed tail), up to the 64-variable cap."""
    from fastbn_amd import synth
    p = str(tmp_path / "s.xml")
    synth.random_network(nv, seed=ns, window=6, dom=(2, 4), path=p)
    cols = synth.forward_sample(synth.read_xmlbif(p), ns, seed=ns + 1)
    dims = np.maximum(cols.max(axis=1).astype(np.int32) + 1, 1)
    assert dims.max() <= 4  # eligible for the device-resident search
    ds = F.Dataset(columns=cols, dims=dims)
    _check(ds, O.OracleDataset(columns=cols, dims=dims), 0.05, 1000, monkeypatch)


def test_dense_graph_hands_off_to_host_at_level_5(monkeypatch):
    """Twelve noisy binary copies of one latent variable, 20k samples: the edges stay dependent
    given any conditioning set, so the search reaches level 5, which the device kernel hands to the
    host driver (levels 0-4 on the device)."""
    rng = np.random.default_rng(7)
    n = 20000
    base = rng.integers(0, 2, n)
    cols = np.stack([base ^ (rng.random(n) < 0.1) for _ in range(12)]).astype(np.uint8)
    dims = np.full(12, 2, np.int32)
    ds = F.Dataset(columns=cols, dims=dims)
    pc = _check(ds, O.OracleDataset(columns=cols, dims=dims), 0.05, 7, monkeypatch)
    assert len(pc.tests_per_level) >= 6


def test_constant_and_two_state_columns(monkeypatch):
    """1-state (constant) columns (df 0: independent) next to 2..4-state ones."""
    rng = np.random.default_rng(3)
    dims = np.array([1, 2, 3, 4, 2, 1, 4, 3], np.int32)
    cols = np.stack([rng.integers(0, d, 6000) for d in dims]).astype(np.uint8)
    cols[2] = (cols[1] + cols[3]) % 3
    cols[6] = (cols[3] + cols[4]) % 4
    ds = F.Dataset(columns=cols, dims=dims)
    _check(ds, O.OracleDataset(columns=cols, dims=dims), 0.05, 1000, monkeypatch)


def test_repeated_runs_and_context_margin_log(alarm):
    """Back-to-back runs on one context reuse its scratch (re-zeroed per launch): identical results;
    the ctx-level margin log afterwards holds the run's log."""
    ds, _ = alarm
    ci = F.IndependenceTest(ds)
    runs = [F.PCStable(0.05, 1000).StructLearnCompData(ci) for _ in range(3)]
    for r in runs[1:]:
        assert r.edges == runs[0].edges and r.sepset == runs[0].sepset
        assert r.tests_per_level.tolist() == runs[0].tests_per_level.tolist()
    m, near = ci.decision_margin()
    assert m == runs[-1].min_margin and near == runs[-1].near_alpha


@pytest.mark.parametrize("mode", ["launch", "timeout"])
def test_fallback_to_host_levels(alarm, mode, monkeypatch):
    """A refused launch, or a grid barrier that times out inside the kernel (a barrier
    limit of one tick), hands the whole search to the host-driven levels: the same tests per level,
    skeleton, sepsets, orientation and SHD as the device-resident path, and a fresh margin log."""
    ds, od = alarm
    dev = F.PCStable(0.05, 1000).StructLearnCompData(ds)
    assert dev.path == 1
    monkeypatch.setenv("FBN_PC_SMALL_FAIL", mode)
    fb = F.PCStable(0.05, 1000).StructLearnCompData(ds)
    monkeypatch.delenv("FBN_PC_SMALL_FAIL")
    assert fb.path == 2
    assert fb.tests_per_level.tolist() == dev.tests_per_level.tolist() == [666, 3579, 828, 118, 15]
    assert fb.edges == dev.edges and fb.sepset == dev.sepset and fb.oriented == dev.oriented
    assert fb.GetSHD(os.path.join(GOLD, "alarm", "alarm.bif")) == 5
    # the host levels' own log (not the failed launch's): the same tests' margins, so no near decisions
    assert fb.near_alpha == 0 and 1e-9 < fb.min_margin < 1.0
    # and the device path works again afterwards (barrier words zeroed again)
    again = F.PCStable(0.05, 1000).StructLearnCompData(ds)
    assert again.path == 1 and again.edges == dev.edges and again.sepset == dev.sepset


def test_cooperative_launch_option(alarm, monkeypatch):
    """FBN_PC_SMALL_COOP=1: the same search through hipLaunchCooperativeKernel (refuses a grid that
    cannot be resident at once); default = plain launch with the bounded-spin fallback."""
    ds, od = alarm
    plain = F.PCStable(0.05, 1000).StructLearnCompData(ds)
    monkeypatch.setenv("FBN_PC_SMALL_COOP", "1")
    coop = F.PCStable(0.05, 1000).StructLearnCompData(ds)
    monkeypatch.delenv("FBN_PC_SMALL_COOP")
    assert plain.path == coop.path == 1
    assert coop.tests_per_level.tolist() == plain.tests_per_level.tolist() == [666, 3579, 828, 118, 15]
    assert coop.edges == plain.edges and coop.sepset == plain.sepset and coop.oriented == plain.oriented
