"""Per-case JT kernel (variant 5, jt_case.hip): one wave per evidence case over the case's
evidence-reduced clique entries, fast arithmetic order (one pass per clique and direction; the
reference's per-multiply normalizations cancel).  Checked against the oracle (the reference's
sequential order) within 1e-12 relative with equal labels, and against the reference's own Munin-like
dump within 1e-9 (north_star allows 1e-6 on potentials)."""
import os

import numpy as np
import pytest
from conftest import GOLD, read_ref_marg

import fastbn_amd as F
import oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-12


@pytest.fixture(scope="module")
def alarm_jt(alarm_paths):
    jt = F.JunctionTree(F.Network(alarm_paths["xml"]), device=0)
    jt.set_variant(5)
    return jt


@pytest.fixture(scope="module")
def alarm_ojt(alarm_paths):
    return O.OracleJT(alarm_paths["xml"])


def _alarm_net():
    from fastbn_amd import synth
    return synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml"))


@pytest.mark.parametrize("which", ["alarm_1k", "alarm_rand"])
def test_case_variant_vs_reference_fixture(alarm_jt, alarm_paths, which):
    path = alarm_paths["test"] if which == "alarm_1k" else alarm_paths["rand"]
    ev, _ = F.load_libsvm(path, 37)
    lab, marg = alarm_jt.infer(ev)
    assert alarm_jt.refresh_info()["variant"] == 5
    rlab, rmarg, _, _ = read_ref_marg(os.path.join(GOLD, which + ".marg.gz"), alarm_jt.network.dims)
    np.testing.assert_array_equal(lab, rlab)
    np.testing.assert_allclose(marg, rmarg, rtol=RTOL, atol=1e-300)


@pytest.mark.parametrize("n,k", [(1, 7), (63, 0), (65, 7), (3000, 12), (2000, 30)])
def test_case_variant_vs_oracle(alarm_jt, alarm_ojt, n, k):
    from fastbn_amd import synth
    ev = synth.evidence_cases(_alarm_net(), n, k, seed=n + k)
    lab, marg = alarm_jt.infer(ev)
    olab, omarg = alarm_ojt.infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_allclose(marg, omarg, rtol=RTOL, atol=1e-300)


def test_case_variant_evidence_extremes_and_fixup(alarm_jt, alarm_ojt):
    rng = np.random.default_rng(3)
    dims = alarm_jt.network.dims
    ev = np.full((130, 37), -1, np.int8)
    ev[1, 1:] = [rng.integers(0, d) for d in dims[1:]]  # everything but the query observed
    ev[2, 1::2] = [rng.integers(0, d) for d in dims[1::2]]
    ev[3, 36] = 0
    ev[70, 1:] = ev[1, 1:]
    lab, marg = alarm_jt.infer(ev)
    olab, omarg = alarm_ojt.infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_allclose(marg, omarg, rtol=RTOL, atol=1e-300)
    alarm_jt.debug_force_fixup(True)  # every block recomputed by the exact interpreter pass
    try:
        lab2, marg2 = alarm_jt.infer(ev)
    finally:
        alarm_jt.debug_force_fixup(False)
    np.testing.assert_array_equal(lab2, olab)
    np.testing.assert_array_equal(marg2, omarg)


@pytest.mark.parametrize("waves,lds", [(1, None), (8, None), (16, "64"), (4, "16384")])
def test_case_variant_geometry(alarm_jt, alarm_ojt, waves, lds, monkeypatch):
    """Waves per CU and the LDS bin budget (FBN_JT_CLDS: 64 sends most bin sets to the global-atomic
    path) change nothing beyond rounding; run to run the results are identical."""
    from fastbn_amd import synth
    if lds is not None:
        monkeypatch.setenv("FBN_JT_CLDS", lds)
    ev = synth.evidence_cases(_alarm_net(), 1500, 9, seed=77)
    olab, omarg = alarm_ojt.infer(ev)
    alarm_jt.set_waves_per_cu(waves)
    try:
        lab, marg = alarm_jt.infer(ev)
        lab2, marg2 = alarm_jt.infer(ev)
    finally:
        alarm_jt.set_waves_per_cu(0)
    np.testing.assert_array_equal(lab2, lab)
    np.testing.assert_array_equal(marg2, marg)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_allclose(marg, omarg, rtol=RTOL, atol=1e-300)


def test_case_variant_synthetic_and_munin_like(tmp_path):
    from fastbn_amd import synth
    for n_nodes, nev, n, seed in ((200, 40, 300, 11), (1041, 208, 136, 1041)):
        p = str(tmp_path / f"syn{n_nodes}.xml")
        synth.random_network(n_nodes, seed=seed, window=10 if n_nodes == 200 else 12, path=p)
        ev = synth.evidence_cases(synth.read_xmlbif(p), n, nev, seed=5)
        ev[0, :] = -1  # no evidence at all
        olab, omarg = O.OracleJT(p).infer(ev)
        jt = F.JunctionTree(F.Network(p), device=0)
        jt.set_variant(5)
        lab, marg = jt.infer(ev)
        np.testing.assert_array_equal(lab, olab)
        np.testing.assert_allclose(marg, omarg, rtol=RTOL, atol=1e-300)


def test_case_variant_munin_fixture_vs_reference(munin_fixture):
    """BASELINE config 4 network: the reference's own 32 fixture cases, labels equal, marginals
    within 1e-9 relative of the reference's dump."""
    jt = F.JunctionTree(F.Network(munin_fixture["xml"]), device=0)
    o = O.OracleJT(munin_fixture["xml"])
    ev, _ = O.load_libsvm(munin_fixture["libsvm"], o.n)
    rlab, rmarg, _, _ = read_ref_marg(munin_fixture["marg"], o.dims)
    jt.set_variant(5)
    lab, marg = jt.infer(ev)
    np.testing.assert_array_equal(lab, rlab)
    np.testing.assert_allclose(marg, rmarg, rtol=1e-9, atol=1e-300)
    olab, omarg = o.infer(ev)
    np.testing.assert_allclose(marg, omarg, rtol=RTOL, atol=1e-300)
