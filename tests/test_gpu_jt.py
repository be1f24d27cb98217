"""Junction-tree HIP path vs the oracle and the reference's own outputs (bit-exact fp64): the exact
arithmetic order (set_exact(True)); the default fast order is tests/test_gpu_jt_fast.py."""
import os

import numpy as np
import pytest
from conftest import GOLD, read_pt_file, read_ref_marg

import fastbn_amd as F
import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def jt(alarm_paths):
    j = F.JunctionTree(F.Network(alarm_paths["xml"]), device=0)
    j.set_exact(True)  # the reference's arithmetic order: bit-identical
    return j


@pytest.fixture(scope="module")
def ojt(alarm_paths):
    return O.OracleJT(alarm_paths["xml"])


@pytest.mark.parametrize("which", ["alarm_1k", "alarm_rand"])
def test_bit_exact_vs_reference_fixture(jt, alarm_paths, which):
    path = alarm_paths["test"] if which == "alarm_1k" else alarm_paths["rand"]
    ev, _ = F.load_libsvm(path, 37)
    lab, marg = jt.infer(ev)
    rlab, rmarg, _, _ = read_ref_marg(os.path.join(GOLD, which + ".marg.gz"), jt.network.dims)
    np.testing.assert_array_equal(lab, rlab)
    np.testing.assert_array_equal(marg, rmarg)


def test_accuracy_and_mse_alarm_1k(jt, alarm_paths):
    ev, gt = F.load_libsvm(alarm_paths["test"], 37)
    gold = read_pt_file(alarm_paths["pt"], jt.network.dims, len(gt))
    acc, mse, hd = jt.EvaluateAccuracy(ev, gt, gold)
    _, _, ref_mse, ref_hd = read_ref_marg(os.path.join(GOLD, "alarm_1k.marg.gz"), jt.network.dims)
    assert acc == 1.0
    assert mse * len(gt) == ref_mse and hd * len(gt) == ref_hd


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000])
def test_ragged_batches_match_oracle(jt, ojt, n):
    from fastbn_amd import synth
    ev = synth.evidence_cases(synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml")), n, 7, seed=n)
    lab, marg = jt.infer(ev)
    olab, omarg = ojt.infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_array_equal(marg, omarg)


def test_evidence_extremes(jt, ojt):
    rng = np.random.default_rng(3)
    dims = jt.network.dims
    ev = np.full((4, 37), -1, np.int8)
    ev[1, 1:] = [rng.integers(0, d) for d in dims[1:]]  # everything but the query observed
    ev[2, 1::2] = [rng.integers(0, d) for d in dims[1::2]]
    ev[3, 36] = 0
    lab, marg = jt.infer(ev)
    olab, omarg = ojt.infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_array_equal(marg, omarg)
    off = np.concatenate([[0], np.cumsum(dims)])
    for v in range(37):  # evidence nodes -> zeros; others -> a distribution
        s = marg[:, off[v]:off[v + 1]].sum(1)
        obs = ev[:, v] >= 0
        assert np.all(s[obs] == 0) and np.allclose(s[~obs], 1.0, atol=1e-12)


def test_large_batch_vs_oracle_and_waves(jt, ojt):
    from fastbn_amd import synth
    net = synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml"))
    ev = synth.evidence_cases(net, 20000, 7, seed=20250131)
    lab, marg = jt.infer(ev)
    olab, omarg = ojt.infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_array_equal(marg, omarg)
    # both kernel variants; LDS variant with and without spilled rows (w=4 -> 80 LDS rows < 144)
    for variant, waves in ((0, 1), (0, 2), (0, 4), (0, 8), (1, 2), (1, 8), (2, 2), (2, 4), (3, 4), (3, 2),
                           (4, 1), (4, 8), (-1, 0)):
        jt.set_variant(variant)
        jt.set_waves_per_cu(waves)
        lab2, marg2 = jt.infer(ev)
        np.testing.assert_array_equal(lab2, lab)
        np.testing.assert_array_equal(marg2, marg)
    jt.set_variant(-1)
    jt.set_waves_per_cu(0)


def test_specialized_kernel_selected_and_fixup(jt, ojt):
    """ALARM is eligible: auto mode runs the plan-specialized kernel (prebuilt code object)."""
    from fastbn_amd import synth
    assert jt.info["specialized_eligible"] == 1
    ev = synth.evidence_cases(synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml")), 3000, 12, seed=3)
    jt.set_variant(-1)
    lab, marg = jt.infer(ev)
    assert jt.refresh_info()["variant"] == 3
    olab, omarg = ojt.infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_array_equal(marg, omarg)
    jt.debug_force_fixup(True)  # every block recomputed by the exact interpreter pass
    lab2, marg2 = jt.infer(ev)
    jt.debug_force_fixup(False)
    np.testing.assert_array_equal(lab2, olab)
    np.testing.assert_array_equal(marg2, omarg)


def test_specialized_synthetic(tmp_path):
    from fastbn_amd import prebuild, synth
    p = prebuild.synth_small_xml(str(tmp_path))
    net = synth.read_xmlbif(p)
    ev = synth.evidence_cases(net, 777, 15, seed=8)
    jt = F.JunctionTree(F.Network(p), device=0)
    jt.set_exact(True)
    assert jt.info["specialized_eligible"] == 1
    olab, omarg = O.OracleJT(p).infer(ev)
    for variant in (3, 0):
        jt.set_variant(variant)
        lab, marg = jt.infer(ev)
        np.testing.assert_array_equal(lab, olab)
        np.testing.assert_array_equal(marg, omarg)


def test_synthetic_network(tmp_path):
    from fastbn_amd import synth
    p = str(tmp_path / "syn.xml")
    synth.random_network(200, seed=11, window=10, path=p)
    net = synth.read_xmlbif(p)
    ev = synth.evidence_cases(net, 300, 40, seed=5)
    jt = F.JunctionTree(F.Network(p), device=0)
    jt.set_exact(True)  # the streamed kernel in the reference's arithmetic order
    olab, omarg = O.OracleJT(p).infer(ev)
    for variant in (0, 1, 2, 4):
        jt.set_variant(variant)
        lab, marg = jt.infer(ev)
        np.testing.assert_array_equal(lab, olab)
        np.testing.assert_array_equal(marg, omarg)


@pytest.mark.parametrize("which", ["alarm_1k", "alarm_rand"])
def test_streamed_variant_vs_reference_fixture(jt, alarm_paths, which):
    """Variant 4 (streamed tables) reproduces the reference's own dump bit for bit, also when every
    block goes through the exact fixup pass."""
    path = alarm_paths["test"] if which == "alarm_1k" else alarm_paths["rand"]
    ev, _ = F.load_libsvm(path, 37)
    rlab, rmarg, _, _ = read_ref_marg(os.path.join(GOLD, which + ".marg.gz"), jt.network.dims)
    jt.set_variant(4)
    try:
        for force in (False, True):
            jt.debug_force_fixup(force)
            lab, marg = jt.infer(ev)
            np.testing.assert_array_equal(lab, rlab)
            np.testing.assert_array_equal(marg, rmarg)
    finally:
        jt.debug_force_fixup(False)
        jt.set_variant(-1)


def test_streamed_variant_munin_like(tmp_path):
    """SURVEY 8(d) config 4 network (seeded Munin-like, 1041 variables, 20 % evidence): the streamed
    kernel and the global interpreter agree with the oracle bit for bit on a ragged batch."""
    from fastbn_amd import synth
    p = str(tmp_path / "munin_like.xml")
    synth.random_network(1041, seed=1041, window=12, path=p, name="munin_like")
    net = synth.read_xmlbif(p)
    ev = synth.evidence_cases(net, 136, 208, seed=20250131)
    ev[0, :] = -1  # no evidence at all
    olab, omarg = O.OracleJT(p).infer(ev)
    jt = F.JunctionTree(F.Network(p), device=0)
    jt.set_exact(True)
    for variant in (4, 1):
        jt.set_variant(variant)
        lab, marg = jt.infer(ev)
        np.testing.assert_array_equal(lab, olab)
        np.testing.assert_array_equal(marg, omarg)
    # the fast arithmetic order (the Munin-class default): within 1e-12 relative, same labels
    jt.set_exact(False)
    jt.set_variant(4)
    lab, marg = jt.infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_allclose(marg, omarg, rtol=1e-12, atol=1e-300)


def test_device_resident_path(jt, ojt):
    torch = pytest.importorskip("torch")
    from fastbn_amd import synth
    ev = synth.evidence_cases(synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml")), 4096, 7, seed=9)
    d_ev = torch.from_numpy(ev).to("cuda")
    d_lab = torch.zeros(4096, dtype=torch.int32, device="cuda")
    d_marg = torch.zeros((4096, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    jt.run_device(d_ev.data_ptr(), 4096, d_lab.data_ptr(), d_marg.data_ptr(), stream)
    torch.cuda.synchronize()
    olab, omarg = ojt.infer(ev)
    np.testing.assert_array_equal(d_lab.cpu().numpy(), olab)
    np.testing.assert_array_equal(d_marg.cpu().numpy(), omarg)


def test_bad_evidence_rejected(jt):
    ev = np.full((2, 37), -1, np.int8)
    ev[1, 5] = 9
    with pytest.raises(F.FastBNError, match="case 1: evidence 9 for node 5"):
        jt.infer(ev)
    ev = np.full((300, 37), -1, np.int8)
    ev[250, 36] = -2
    ev[299, 0] = 7
    with pytest.raises(F.FastBNError, match="case 250: evidence -2 for node 36"):  # the first one
        jt.infer(ev)
    ev[250, 36] = -1
    ev[299, 0] = -1
    lab, _ = jt.infer(ev)  # the plan stays usable after a rejected batch
    assert lab.shape == (300,)


def test_bad_evidence_rejected_on_device_path(jt, ojt):
    """fbn_jt_run_device checks a device buffer's codes by default (FBN_ERR_ARG naming the first bad
    case/node); fbn_jt_evidence_validate is the check alone; with the check off the run is
    asynchronous and a valid buffer gives the oracle's results."""
    torch = pytest.importorskip("torch")
    from fastbn_amd import synth
    n = 512
    ev = synth.evidence_cases(synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml")), n, 7, seed=11)
    bad = ev.copy()
    bad[300, 12] = 5  # node 12 has fewer states
    bad[400, 3] = -3
    d_bad = torch.from_numpy(bad).to("cuda")
    d_lab = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_marg = torch.zeros((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    with pytest.raises(F.FastBNError, match="case 300: evidence 5 for node 12"):
        jt.run_device(d_bad.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), stream)
    with pytest.raises(F.FastBNError, match="case 300: evidence 5 for node 12"):
        jt.validate_device(d_bad.data_ptr(), n, stream)
    d_ev = torch.from_numpy(ev).to("cuda")
    jt.validate_device(d_ev.data_ptr(), n, stream)
    jt.set_evidence_check(False)
    try:
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), stream)
        torch.cuda.synchronize()
    finally:
        jt.set_evidence_check(True)
    olab, omarg = ojt.infer(ev)
    np.testing.assert_array_equal(d_lab.cpu().numpy(), olab)
    np.testing.assert_array_equal(d_marg.cpu().numpy(), omarg)


def test_munin_like_full_network_vs_reference(munin_fixture):
    """BASELINE config 4 at its real network size on the reference's 32 fixture cases: the tiled
    kernel (default for the 1041-variable plan, fast order) -- labels equal to the reference's,
    marginals within 1e-9 relative; the streamed kernel in exact order -- within 1e-12 relative (the
    reference's heap-ordered tree breaks a few Prim ties differently, conftest.MUNIN_REF_RTOL) and
    bit-identical to the restatement on our tree."""
    from conftest import MUNIN_REF_RTOL, read_ref_marg
    jt = F.JunctionTree(F.Network(munin_fixture["xml"]), device=0)
    o = O.OracleJT(munin_fixture["xml"])
    ev, _ = O.load_libsvm(munin_fixture["libsvm"], o.n)
    rlab, rmarg, _, _ = read_ref_marg(munin_fixture["marg"], o.dims)
    olab, omarg = o.infer(ev)
    # default (auto = fast order for this plan, the tiled kernel): labels equal the reference's,
    # marginals within 1e-9 relative of the reference's own (north_star: 1e-6)
    lab, marg = jt.infer(ev)
    assert jt.refresh_info()["variant"] == 5
    np.testing.assert_array_equal(lab, rlab)
    np.testing.assert_allclose(marg, rmarg, rtol=1e-9, atol=1e-300)
    np.testing.assert_allclose(marg, omarg, rtol=1e-12, atol=1e-300)
    # exact order: bit-identical to the restatement on our tree, 1e-12 of the reference's
    jt.set_exact(True)
    lab, marg = jt.infer(ev)
    np.testing.assert_array_equal(lab, rlab)
    np.testing.assert_allclose(marg, rmarg, rtol=MUNIN_REF_RTOL, atol=1e-300)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_array_equal(marg, omarg)


def test_munin_like_extra_cases_vs_reference(munin_fixture):
    """The default Munin-class path (tiled kernel, fast order) on 64 more reference cases at 0 / 52 /
    208 / 520 observed variables: labels equal the reference's, marginals within 1e-9 relative,
    nothing handed to the exact fixup."""
    from conftest import read_ref_marg
    jt = F.JunctionTree(F.Network(munin_fixture["xml"]), device=0)
    o = O.OracleJT(munin_fixture["xml"])
    ev, _ = O.load_libsvm(munin_fixture["extra_libsvm"], o.n)
    rlab, rmarg, _, _ = read_ref_marg(munin_fixture["extra_marg"], o.dims)
    lab, marg = jt.infer(ev)
    assert jt.refresh_info()["variant"] == 5 and jt.debug_flagged_blocks() == 0
    np.testing.assert_array_equal(lab, rlab)
    np.testing.assert_allclose(marg, rmarg, rtol=1e-9, atol=1e-300)


def test_network_from_counts_runs_like_xmlbif():
    """A network handed over in memory (fbn_network_create) infers exactly like the XMLBIF path:
    labels and marginals bit for bit, fast and exact order."""
    from test_host import _counts_from_xmlbif
    from fastbn_amd import synth
    xml = os.path.join(GOLD, "alarm", "alarm.xml")
    names, dims, parents, counts = _counts_from_xmlbif(xml)
    ev = synth.evidence_cases(synth.read_xmlbif(xml), 2000, 7, seed=31)
    a = F.JunctionTree(F.Network.from_counts(dims, parents, counts, names), device=0)
    b = F.JunctionTree(F.Network(xml), device=0)
    for exact in (None, True):
        a.set_exact(exact)
        b.set_exact(exact)
        la, ma = a.infer(ev)
        lb, mb = b.infer(ev)
        np.testing.assert_array_equal(la, lb)
        np.testing.assert_array_equal(ma, mb)
