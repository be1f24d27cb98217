"""The variable-major output layout of fbn_jt_run_device (fbn_jt_set_output_layout(p, 1): marginals
[sum_dom][ncases]) and the device-side scoring terms (fbn_jt_score_terms_device).

Every kernel variant gives the same values in both layouts: the specialized kernel (3) stores the
variable-major columns itself (and so does its exact fixup pass), the interpreters (0 / 1) take a
column stride, the streamed (4) and tiled (5) kernels write case-major scratch that is transposed
into place.  The reference's own per-case vectors (GetProbabilitiesAllNodes, src/JunctionTree.cpp:
1385-1454) are the case-major rows; the checks below compare bit for bit.  The per-case MSE / HD terms
summed in case order equal fbn_jt_score and the reference's own sums (src/Inference.cpp:153-206)."""
import os

import numpy as np
import pytest
from conftest import GOLD, read_pt_file, read_ref_marg

import fastbn_amd as F
import oracle as O
from fastbn_amd import synth

pytestmark = pytest.mark.gpu
XML = os.path.join(GOLD, "alarm", "alarm.xml")


def _run(jt, ev, layout):
    """run_device on torch buffers -> (labels, marginals as case-major numpy)."""
    import torch
    dev = torch.device("cuda", 0)
    n, SD = ev.shape[0], jt.info["sum_dom"]
    d_ev = torch.from_numpy(np.ascontiguousarray(ev)).to(dev)
    d_lab = torch.full((n,), -7, dtype=torch.int32, device=dev)
    d_marg = torch.full((n * SD,), float("nan"), dtype=torch.float64, device=dev)
    jt.set_output_layout(layout)
    try:
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(),
                      torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
    finally:
        jt.set_output_layout(0)
    m = d_marg.view(SD, n).t() if layout == 1 else d_marg.view(n, SD)
    return d_lab.cpu().numpy(), m.cpu().numpy()


@pytest.fixture(scope="module")
def alarm_jt():
    return F.JunctionTree(F.Network(XML), device=0)


@pytest.mark.parametrize("variant,exact", [(3, None), (3, True), (0, True), (1, True), (4, True), (4, None),
                                           (5, None)])
@pytest.mark.parametrize("n", [1, 65, 1000])
def test_variable_major_equals_case_major(alarm_jt, variant, exact, n):
    ev = synth.evidence_cases(synth.read_xmlbif(XML), n, 7, seed=100 + n)
    alarm_jt.set_variant(variant)
    alarm_jt.set_exact(exact)
    try:
        lab0, m0 = _run(alarm_jt, ev, 0)
        lab1, m1 = _run(alarm_jt, ev, 1)
    finally:
        alarm_jt.set_variant(-1)
        alarm_jt.set_exact(None)
    np.testing.assert_array_equal(lab1, lab0)
    np.testing.assert_array_equal(m1, m0)
    olab, omarg = O.OracleJT(XML).infer(ev)
    np.testing.assert_array_equal(lab1, olab)
    if exact:
        np.testing.assert_array_equal(m1, omarg)
    else:
        np.testing.assert_allclose(m1, omarg, rtol=1e-12, atol=1e-300)


def test_variable_major_fixup_pass(alarm_jt):
    """Every block forced through the exact fixup pass (LDS interpreter) in the variable-major layout."""
    ev = synth.evidence_cases(synth.read_xmlbif(XML), 333, 9, seed=5)
    olab, omarg = O.OracleJT(XML).infer(ev)
    alarm_jt.debug_force_fixup(True)
    try:
        lab, m = _run(alarm_jt, ev, 1)
    finally:
        alarm_jt.debug_force_fixup(False)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_allclose(m, omarg, rtol=1e-12, atol=1e-300)


def test_variable_major_munin_like_tiled(munin_fixture):
    """The tiled kernel (variant 5, Munin-class default) through the transpose: the reference's own
    labels and marginals (1e-9: its Prim ties)."""
    jt = F.JunctionTree(F.Network(munin_fixture["xml"]), device=0)
    ev, _ = F.load_libsvm(munin_fixture["libsvm"], jt.info["num_nodes"])
    lab0, m0 = _run(jt, ev, 0)
    lab1, m1 = _run(jt, ev, 1)
    assert jt.refresh_info()["variant"] == 5
    np.testing.assert_array_equal(lab1, lab0)
    np.testing.assert_array_equal(m1, m0)
    rlab, rmarg, _, _ = read_ref_marg(munin_fixture["marg"], jt.network.dims)
    np.testing.assert_array_equal(lab1, rlab)
    np.testing.assert_allclose(m1, rmarg, rtol=1e-9, atol=1e-300)


@pytest.mark.parametrize("layout", [0, 1])
def test_score_terms_device_equal_host_score_and_reference(alarm_paths, layout):
    """Device terms of the reference's alarm_1k test set (exact order), summed in case order: equal to
    fbn_jt_score on the host and to the reference's own MSE / HD sums, bit for bit."""
    import torch
    dev = torch.device("cuda", 0)
    jt = F.JunctionTree(F.Network(alarm_paths["xml"]), device=0)
    jt.set_exact(True)
    ev, gt = F.load_libsvm(alarm_paths["test"], 37)
    n, SD = len(gt), jt.info["sum_dom"]
    gold = read_pt_file(alarm_paths["pt"], jt.network.dims, n)
    d_ev = torch.from_numpy(ev).to(dev)
    d_lab = torch.empty(n, dtype=torch.int32, device=dev)
    d_marg = torch.empty(n * SD, dtype=torch.float64, device=dev)
    d_gold = torch.from_numpy(np.ascontiguousarray(gold)).to(dev)
    d_terms = torch.empty(2 * n, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    jt.set_output_layout(layout)
    jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), s)
    jt.score_terms_device(d_marg.data_ptr(), d_gold.data_ptr(), n, d_terms.data_ptr(), s)
    torch.cuda.synchronize(dev)
    terms = d_terms.cpu().numpy().reshape(n, 2)
    mse = hd = 0.0
    for c in range(n):  # case order, as fbn_jt_score / Inference::EvaluateAccuracy
        mse += float(terms[c, 0])
        hd += float(terms[c, 1])
    _, marg = jt.infer(ev)
    hmse, hhd = jt.score(marg, gold)
    _, _, ref_mse, ref_hd = read_ref_marg(os.path.join(GOLD, "alarm_1k.marg.gz"), jt.network.dims)
    assert mse == hmse and hd == hhd
    assert mse == ref_mse and hd == ref_hd


def test_output_layout_rejects_bad_value(alarm_jt):
    with pytest.raises(F.FastBNError):
        alarm_jt.set_output_layout(2)
