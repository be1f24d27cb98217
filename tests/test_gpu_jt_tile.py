"""The tiled JT kernel (variant 5, fastbn_amd/csrc/jt_tile.hip: 16 cases x 4 entry slots per wave,
fast arithmetic order -- the Munin-class default) against the oracle: labels equal, marginals within
1e-12 relative (north_star allows 1e-6 on potentials), evidence variables zero, every other marginal a
distribution; the forced exact-fixup path bit-identical to the oracle; run-to-run identical results.
The reference's own Munin-like dump: tests/test_gpu_jt.py::test_munin_like_full_network_vs_reference."""
import os

import numpy as np
import pytest
from conftest import GOLD

import fastbn_amd as F
import oracle as O
from fastbn_amd import synth

pytestmark = pytest.mark.gpu
ALARM = os.path.join(GOLD, "alarm", "alarm.xml")


def _check(lab, marg, olab, omarg, ev, dims):
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_allclose(marg, omarg, rtol=1e-12, atol=1e-300)
    off = np.concatenate([[0], np.cumsum(dims)])
    for v in range(len(dims)):
        s = marg[:, off[v]:off[v + 1]].sum(1)
        obs = ev[:, v] >= 0
        assert np.all(marg[obs, off[v]:off[v + 1]] == 0) and np.allclose(s[~obs], 1.0, atol=1e-12)


@pytest.fixture(scope="module")
def alarm():
    jt = F.JunctionTree(F.Network(ALARM), device=0)
    assert jt.info["tiled_eligible"] == 1
    jt.set_variant(5)
    return jt, O.OracleJT(ALARM)


@pytest.mark.parametrize("n", [1, 15, 16, 17, 63, 64, 65, 1000])
def test_alarm_ragged_batches(alarm, n):
    jt, ojt = alarm
    ev = synth.evidence_cases(synth.read_xmlbif(ALARM), n, 7, seed=100 + n)
    lab, marg = jt.infer(ev)
    assert jt.debug_flagged_blocks() == 0  # the tiled kernel's own results (no exact recomputation)
    _check(lab, marg, *ojt.infer(ev), ev, jt.network.dims)


def test_alarm_evidence_extremes(alarm):
    jt, ojt = alarm
    rng = np.random.default_rng(5)
    dims = jt.network.dims
    ev = np.full((20, 37), -1, np.int8)
    ev[1, 1:] = [rng.integers(0, d) for d in dims[1:]]  # everything but the query observed
    ev[2, 1::2] = [rng.integers(0, d) for d in dims[1::2]]
    ev[3, 36] = 0
    for r in range(4, 20):  # many observed variables, random
        k = rng.integers(1, 30)
        vs = rng.choice(np.arange(1, 37), k, replace=False)
        ev[r, vs] = [rng.integers(0, dims[v]) for v in vs]
    lab, marg = jt.infer(ev)
    _check(lab, marg, *ojt.infer(ev), ev, dims)


def test_alarm_forced_fixup_is_exact(alarm):
    """Every 64-case block through the exact interpreter pass: the oracle's bits."""
    jt, ojt = alarm
    ev = synth.evidence_cases(synth.read_xmlbif(ALARM), 300, 7, seed=4)
    jt.debug_force_fixup(True)
    try:
        lab, marg = jt.infer(ev)
    finally:
        jt.debug_force_fixup(False)
    olab, omarg = ojt.infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_array_equal(marg, omarg)


def test_run_to_run_identical_and_waves(alarm):
    jt, _ = alarm
    ev = synth.evidence_cases(synth.read_xmlbif(ALARM), 5000, 7, seed=6)
    lab, marg = jt.infer(ev)
    for w in (4, 8, 16, 0):
        jt.set_waves_per_cu(w)
        lab2, marg2 = jt.infer(ev)
        np.testing.assert_array_equal(lab2, lab)
        np.testing.assert_array_equal(marg2, marg)


@pytest.mark.parametrize("nodes,window,dom,k", [(200, 10, (2, 5), 40), (120, 6, (2, 8), 25), (60, 4, (5, 8), 10)])
def test_synthetic_networks(tmp_path, nodes, window, dom, k):
    """Random networks, state counts up to 8 (the marginal sweep's value chunks > 4 slots)."""
    p = str(tmp_path / "syn.xml")
    synth.random_network(nodes, seed=nodes + k, window=window, dom=dom, path=p)
    net = synth.read_xmlbif(p)
    ev = synth.evidence_cases(net, 333, k, seed=nodes)
    ev[0, :] = -1  # no evidence
    jt = F.JunctionTree(F.Network(p), device=0)
    if not jt.info["tiled_eligible"]:
        pytest.skip("plan outside the tiled variant's limits")
    jt.set_variant(5)
    lab, marg = jt.infer(ev)
    assert jt.debug_flagged_blocks() == 0
    _check(lab, marg, *O.OracleJT(p).infer(ev), ev, jt.network.dims)


def test_munin_like_default_and_vs_oracle(tmp_path):
    """BASELINE config 4's network: auto mode takes the tiled kernel (fast order); 136 cases incl. one
    without evidence against the oracle; exact mode still runs the streamed kernel (variant 4)."""
    p = str(tmp_path / "munin_like.xml")
    synth.random_network(1041, seed=1041, window=12, path=p, name="munin_like")
    net = synth.read_xmlbif(p)
    ev = synth.evidence_cases(net, 136, 208, seed=20250131)
    ev[0, :] = -1
    jt = F.JunctionTree(F.Network(p), device=0)
    lab, marg = jt.infer(ev)
    assert jt.refresh_info()["variant"] == 5
    assert jt.debug_flagged_blocks() == 0
    olab, omarg = O.OracleJT(p).infer(ev)
    _check(lab, marg, olab, omarg, ev, jt.network.dims)
    jt.set_exact(True)
    lab, marg = jt.infer(ev)
    assert jt.refresh_info()["variant"] == 4
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_array_equal(marg, omarg)


@pytest.mark.parametrize("k", [104, 416])
def test_munin_like_large_batch_spread_vs_oracle(tmp_path, k):
    """16,384 Munin-like cases in one launch at 10 % / 40 % evidence (the bench's shape at full
    occupancy: 1,024 case groups): the oracle on 160 cases spread over the batch (the last
    included), and every case through bench.jt_full_batch_properties (rows sum to 1, evidence rows
    zero, each label the first strict maximum of variable 0's marginal)."""
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    p = str(tmp_path / "munin_like.xml")
    synth.random_network(1041, seed=1041, window=12, path=p, name="munin_like")
    n = 16384
    ev = synth.evidence_cases(synth.read_xmlbif(p), n, k, seed=7 + k)
    jt = F.JunctionTree(F.Network(p), device=0)
    lab, marg = jt.infer(ev)
    assert jt.refresh_info()["variant"] == 5
    pick = bench.oracle_sample(n, 1, 160)
    olab, omarg = O.OracleJT(p).infer(ev[pick])
    _check(lab[pick], marg[pick], olab, omarg, ev[pick], jt.network.dims)
    props = bench.jt_full_batch_properties(torch.from_numpy(ev), torch.from_numpy(lab), torch.from_numpy(marg),
                                           jt.network.dims)
    assert props["ok"] and props["cases"] == n, props


def test_loop_tiled_munin_like_vs_reference(munin_fixture, monkeypatch):
    """FBN_JT_TILING = 1 (opt-in loop tiling: chunk-major R streams, bins written by a run's first
    chunk and added into by the later ones) on the reference's own Munin-like fixture cases."""
    from conftest import read_ref_marg
    monkeypatch.setenv("FBN_JT_TILING", "1")
    jt = F.JunctionTree(F.Network(munin_fixture["xml"]), device=0)
    o = O.OracleJT(munin_fixture["xml"])
    ev, _ = O.load_libsvm(munin_fixture["libsvm"], o.n)
    rlab, rmarg, _, _ = read_ref_marg(munin_fixture["marg"], o.dims)
    lab, marg = jt.infer(ev)
    assert jt.refresh_info()["variant"] == 5
    np.testing.assert_array_equal(lab, rlab)
    np.testing.assert_allclose(marg, rmarg, rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(marg, o.infer(ev)[1], rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize("tw", [2, 4])
def test_multi_wave_case_groups(alarm, tmp_path, monkeypatch, tw):
    """FBN_JT_TW = 2 / 4 waves per case group (opt-in: passes split over the waves, one LDS stage
    per case group): ALARM and a synthetic network against the oracle, nothing flagged."""
    monkeypatch.setenv("FBN_JT_TW", str(tw))
    _, ojt = alarm
    jt = F.JunctionTree(F.Network(ALARM), device=0)
    jt.set_variant(5)
    ev = synth.evidence_cases(synth.read_xmlbif(ALARM), 777, 7, seed=tw)
    lab, marg = jt.infer(ev)
    assert jt.debug_flagged_blocks() == 0
    _check(lab, marg, *ojt.infer(ev), ev, jt.network.dims)
    p = str(tmp_path / "syn.xml")
    synth.random_network(200, seed=200 + tw, window=10, path=p)
    ev = synth.evidence_cases(synth.read_xmlbif(p), 333, 40, seed=tw)
    jt = F.JunctionTree(F.Network(p), device=0)
    jt.set_variant(5)
    lab, marg = jt.infer(ev)
    assert jt.debug_flagged_blocks() == 0
    _check(lab, marg, *O.OracleJT(p).infer(ev), ev, jt.network.dims)


@pytest.mark.parametrize("name", ["bigdom", "wide"])
def test_synth_nets_default_path_vs_reference(synth_nets, name):
    """Through the default path (auto: the tiled kernel, fast order): a network with state counts up
    to 21 and one with a 12-variable clique (evidence on clique variables past the 10th), against the
    reference's own labels and marginals (tests/golden/synth_nets; 1e-9 as for the Munin-like dumps:
    bigdom's tree breaks Prim ties differently) and the oracle (1e-12); nothing flagged for the exact
    pass unless a query marginal is a near-tie."""
    fx = synth_nets[name]
    jt = F.JunctionTree(F.Network(fx["xml"]), device=0)
    lab, marg = jt.infer(fx["ev"])
    assert jt.refresh_info()["variant"] == 5
    np.testing.assert_array_equal(lab, fx["labels"])
    np.testing.assert_allclose(marg, fx["marg"], rtol=1e-9, atol=1e-300)
    _check(lab, marg, *O.OracleJT(fx["xml"]).infer(fx["ev"]), fx["ev"], fx["dims"])
    # more cases, random evidence incl. every variable of the wide clique observed
    net = synth.read_xmlbif(fx["xml"])
    ev = synth.evidence_cases(net, 300, len(fx["dims"]) // 3, seed=99)
    ev[:8] = synth.evidence_cases(net, 8, len(fx["dims"]) - 1, seed=98)
    lab, marg = jt.infer(ev)
    _check(lab, marg, *O.OracleJT(fx["xml"]).infer(ev), ev, fx["dims"])


@pytest.mark.parametrize("variant", [None, 5, 4])
def test_tied_query_marginals_label_like_reference(synth_nets, variant):
    """Symmetric CPTs: X0's posterior ties exactly in 24 of the 64 fixture cases.  The fast arithmetic
    order (default; kernels 3 / 5 / 4) flags a block whose top two query values are within 1e-12 and
    the exact pass recomputes it, so labels equal the reference's ArgMax (strict '>' from 0) on every
    tie (near-tie label stability)."""
    fx = synth_nets["tie"]
    jt = F.JunctionTree(F.Network(fx["xml"]), device=0)
    if variant is not None:
        jt.set_variant(variant)
    lab, marg = jt.infer(fx["ev"])
    assert jt.refresh_info()["variant"] == (variant if variant is not None else 3)
    np.testing.assert_array_equal(lab, fx["labels"])
    np.testing.assert_allclose(marg, fx["marg"], rtol=1e-12, atol=1e-300)
    assert jt.debug_flagged_blocks() >= 1  # the ties went through the exact pass
