"""The default (fast) arithmetic order of the plan-specialized ALARM-class kernel (variant 3,
jt_codegen.cpp): a clique's table is its initial potential times its messages, normalized once
where a message or marginal is formed -- the reference's intermediate normalizations
(src/JunctionTree.cpp:829-941, 1150-1238) cancel.  Labels equal the reference's own dumps and the
oracle; marginals within 1e-12 relative (north_star allows 1e-6)."""
import os

import numpy as np
import pytest
from conftest import GOLD, read_ref_marg

import fastbn_amd as F
import oracle as O
from fastbn_amd import prebuild, synth

pytestmark = pytest.mark.gpu
TOL = 1e-12


def _close(marg, ref):
    np.testing.assert_allclose(marg, ref, rtol=TOL, atol=1e-300)


@pytest.fixture(scope="module")
def jt(alarm_paths):
    j = F.JunctionTree(F.Network(alarm_paths["xml"]), device=0)
    j.set_exact(None)  # auto = fast
    return j


@pytest.mark.parametrize("which", ["alarm_1k", "alarm_rand"])
def test_fast_vs_reference_fixture(jt, alarm_paths, which):
    path = alarm_paths["test"] if which == "alarm_1k" else alarm_paths["rand"]
    ev, _ = F.load_libsvm(path, 37)
    lab, marg = jt.infer(ev)
    assert jt.refresh_info()["variant"] == 3
    rlab, rmarg, _, _ = read_ref_marg(os.path.join(GOLD, which + ".marg.gz"), jt.network.dims)
    np.testing.assert_array_equal(lab, rlab)
    _close(marg, rmarg)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 20000])
def test_fast_ragged_vs_oracle(jt, n):
    net = synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml"))
    ev = synth.evidence_cases(net, n, 7, seed=n)
    lab, marg = jt.infer(ev)
    assert jt.debug_flagged_blocks() == 0  # the specialized kernel's own results
    olab, omarg = O.OracleJT(os.path.join(GOLD, "alarm", "alarm.xml")).infer(ev)
    np.testing.assert_array_equal(lab, olab)
    _close(marg, omarg)


def test_fast_evidence_extremes_and_fixup(jt):
    rng = np.random.default_rng(3)
    dims = jt.network.dims
    ev = np.full((130, 37), -1, np.int8)
    ev[1, 1:] = [rng.integers(0, d) for d in dims[1:]]  # everything but the query observed
    ev[2, 1::2] = [rng.integers(0, d) for d in dims[1::2]]
    ev[3, 36] = 0
    ev[4:] = synth.evidence_cases(synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml")), 126, 20, seed=9)
    olab, omarg = O.OracleJT(os.path.join(GOLD, "alarm", "alarm.xml")).infer(ev)
    for force in (False, True):  # True: every block recomputed by the exact interpreter pass
        jt.debug_force_fixup(force)
        lab, marg = jt.infer(ev)
        np.testing.assert_array_equal(lab, olab)
        _close(marg, omarg)
    jt.debug_force_fixup(False)
    off = np.concatenate([[0], np.cumsum(dims)])
    for v in range(37):  # evidence nodes -> zeros; others -> a distribution
        s = marg[:, off[v]:off[v + 1]].sum(1)
        obs = ev[:, v] >= 0
        assert np.all(s[obs] == 0) and np.allclose(s[~obs], 1.0, atol=1e-12)


def test_fast_and_exact_kernels_switch(jt):
    """Toggling the order reloads the matching code object; exact stays bit-identical."""
    net = synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml"))
    ev = synth.evidence_cases(net, 500, 7, seed=4)
    olab, omarg = O.OracleJT(os.path.join(GOLD, "alarm", "alarm.xml")).infer(ev)
    try:
        for exact in (True, False, True):
            jt.set_exact(exact)
            lab, marg = jt.infer(ev)
            assert jt.refresh_info()["variant"] == 3
            np.testing.assert_array_equal(lab, olab)
            if exact:
                np.testing.assert_array_equal(marg, omarg)
            else:
                _close(marg, omarg)
    finally:
        jt.set_exact(None)


def test_fast_specialized_synthetic(tmp_path):
    from fastbn_amd import prebuild
    p = prebuild.synth_small_xml(str(tmp_path))
    ev = synth.evidence_cases(synth.read_xmlbif(p), 777, 15, seed=8)
    jt = F.JunctionTree(F.Network(p), device=0)
    assert jt.info["specialized_eligible"] == 1
    jt.set_variant(3)
    lab, marg = jt.infer(ev)
    olab, omarg = O.OracleJT(p).infer(ev)
    np.testing.assert_array_equal(lab, olab)
    _close(marg, omarg)


@pytest.mark.parametrize("env", prebuild.ALARM_TEST_OPTIONS)
def test_fast_codegen_options_vs_reference(alarm_paths, monkeypatch, env):
    """Code-generation options of the fast order against the reference's own ALARM dump: leaf
    Collect messages recomputed in the parent's Distribute (opt-in), no LDS message pool (every
    message in the per-wave global rows), and the branched marginal stores -- each changes where a
    message lives or how a marginal is stored, never the values (labels equal, <= 1e-12)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    j = F.JunctionTree(F.Network(alarm_paths["xml"]), device=0)
    j.set_variant(3)
    ev, _ = F.load_libsvm(alarm_paths["rand"], 37)
    lab, marg = j.infer(ev)
    assert j.debug_flagged_blocks() == 0
    rlab, rmarg, _, _ = read_ref_marg(os.path.join(GOLD, "alarm_rand.marg.gz"), j.network.dims)
    np.testing.assert_array_equal(lab, rlab)
    _close(marg, rmarg)


def test_kernel_timing_switch(jt):
    """fbn_jt_set_kernel_timing(0): no timing events (last_kernel_ms raises), identical results."""
    ev = synth.evidence_cases(synth.read_xmlbif(os.path.join(GOLD, "alarm", "alarm.xml")), 5000, 7, seed=11)
    lab0, marg0 = jt.infer(ev)
    assert jt.last_kernel_ms() > 0
    jt.set_kernel_timing(False)
    try:
        lab1, marg1 = jt.infer(ev)
        with pytest.raises(F.FastBNError):
            jt.last_kernel_ms()
    finally:
        jt.set_kernel_timing(True)
    np.testing.assert_array_equal(lab0, lab1)
    np.testing.assert_array_equal(marg0, marg1)


def test_headline_size_100k_default_and_exact(jt):
    """BASELINE config 2 at its real size through the bench's path: 100,000 ALARM cases (1,563
    64-case blocks: two rounds on 1,024 SIMDs, the 539-block tail included) in device buffers
    (fbn_jt_run_device).  Default (fast) order: labels equal and marginals within 1e-12 of the
    oracle on 2,048+ cases spread over the batch (the last block included), and every case passes
    bench.jt_full_batch_properties.  Exact order on the same batch: bit-identical to the oracle on
    the sample (src/JunctionTree.cpp:1508-1534, src/Inference.cpp:92-102)."""
    import torch
    import bench  # (conftest puts the repo root on sys.path)
    n = 100_000
    xml = os.path.join(GOLD, "alarm", "alarm.xml")
    ev = jt.network.evidence_cases(n, 7, 20250131)
    dev = torch.device("cuda", 0)
    d_ev = torch.from_numpy(ev).to(dev)
    d_lab = torch.empty(n, dtype=torch.int32, device=dev)
    d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    pick = bench.oracle_sample(n, 256, 1792)
    pick = np.unique(np.concatenate([pick, np.arange(n - 64, n)]))  # the whole last block
    olab, omarg = O.OracleJT(xml).infer(ev[pick])
    ip = torch.from_numpy(pick).to(dev)
    try:
        for exact in (None, True):
            jt.set_exact(exact)
            d_lab.fill_(-7)
            d_marg.fill_(np.nan)
            jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), stream)
            torch.cuda.synchronize(dev)
            assert jt.refresh_info()["variant"] == 3
            lab, marg = d_lab[ip].cpu().numpy(), d_marg[ip].cpu().numpy()
            np.testing.assert_array_equal(lab, olab)
            if exact:
                np.testing.assert_array_equal(marg, omarg)
            else:
                assert jt.debug_flagged_blocks() == 0
                _close(marg, omarg)
            props = bench.jt_full_batch_properties(d_ev, d_lab, d_marg, jt.network.dims)
            assert props["ok"] and props["cases"] == n and props["label_near_ties"] == 0, props
    finally:
        jt.set_exact(None)
