"""The tiled kernel's program (variant 5: jt_tile_plan.cpp -> jt_tile.hip) executed on the host by
tests/tile_emulator.py (numpy, the kernel's algebra) against the oracle and the reference's own
outputs: the G / R index records, factor offsets, LDS staging records, partial / output bins and the
static marginal sources are checked without a GPU.  The GPU kernel itself: tests/test_gpu_jt.py."""
import os

import numpy as np
from conftest import GOLD

import fastbn_amd as F
import oracle as O
import tile_emulator as TE
from fastbn_amd import synth

ALARM = os.path.join(GOLD, "alarm", "alarm.xml")


def _prog(xml):
    jt = F.JunctionTree(F.Network(xml), device=-1)  # host-only plan: no GPU needed
    assert jt.info["tiled_eligible"] == 1
    return jt, jt.tile_program()


def test_alarm_random_evidence_vs_oracle():
    jt, prog = _prog(ALARM)
    ev = synth.evidence_cases(synth.read_xmlbif(ALARM), 96, 7, seed=3)
    lab, marg = TE.run(prog, ev, jt.info["sum_dom"])
    olab, omarg = O.OracleJT(ALARM).infer(ev)
    np.testing.assert_array_equal(lab, olab)
    np.testing.assert_allclose(marg, omarg, rtol=1e-12, atol=0)


def test_every_pass_covers_its_clique_once():
    """G x R of every pass enumerates each entry of its clique exactly once; partial-bin indices
    cover [0, nbins * nE) exactly once."""
    for xml in (ALARM,):
        jt, (passes, tab, iv, geo) = _prog(xml)
        for prow in passes:
            P = dict(zip(TE.F, (int(x) for x in prow)))
            nf, nG, nRo, nRi = P["nf"], P["nG"], P["nRo"], P["nRi"]
            g = tab[P["g_off"]:P["g_off"] + nG * (4 + nf)].reshape(nG, 4 + nf).astype(np.int64)
            ro = tab[P["o_off"]:P["o_off"] + nRo * (4 + nf)].reshape(nRo, 4 + nf).astype(np.int64)
            ri = tab[P["i_off"]:P["i_off"] + nRi * (2 + nf)].reshape(nRi, 2 + nf).astype(np.int64)
            er = (ro[:, 0:1] + ri[None, :, 0] // 8).reshape(-1)
            e = (g[:, 0:1] + er[None, :]).reshape(-1)
            assert sorted(e.tolist()) == list(range(nG * nRo * nRi))
            x = (g[:, 2:3] + ro[None, :, 2]).reshape(-1)
            assert sorted(x.tolist()) == list(range(P["nbins"] * P["nE"]))
            assert P["rounds"] * geo["slots"] >= nG


def test_munin_like_fixture_vs_reference(munin_fixture):
    """The seeded Munin-like network (1041 variables) on the reference's own dump (tests/golden/
    munin_like, oracle/_ref/ref_dump jt): labels equal, marginals within 1e-9 relative."""
    from conftest import read_ref_marg
    jt, prog = _prog(munin_fixture["xml"])
    o = O.OracleJT(munin_fixture["xml"])
    ev, _ = O.load_libsvm(munin_fixture["libsvm"], o.n)
    rlab, rmarg, _, _ = read_ref_marg(munin_fixture["marg"], o.dims)
    n = 8  # (the emulator runs ~0.2 s per case)
    lab, marg = TE.run(prog, ev[:n], jt.info["sum_dom"])
    np.testing.assert_array_equal(lab, rlab[:n])
    np.testing.assert_allclose(marg, rmarg[:n], rtol=1e-9, atol=1e-300)


def _check_steps(passes, tab, geo):
    """The flattened step records the kernel reads equal the outer x inner composition, with bit 0 of a
    factor soffset set exactly where the row equals the step before's; chunk padding present."""
    C = geo["cases_per_wave"]
    for prow in passes:
        P = dict(zip(TE.F, (int(x) for x in prow)))
        nf, nRo, nRi = P["nf"], P["nRo"], P["nRi"]
        nR = nRo * nRi
        assert 0 <= P["nl"] <= nf
        ro = tab[P["o_off"]:P["o_off"] + nRo * (4 + nf)].reshape(nRo, 4 + nf).astype(np.int64)
        ri = tab[P["i_off"]:P["i_off"] + nRi * (2 + nf)].reshape(nRi, 2 + nf).astype(np.int64)
        et = tab[P["et_off"]:P["et_off"] + nR + C].astype(np.int64)
        st = tab[P["st_off"]:P["st_off"] + (nR + C) * (nf + 2)].reshape(nR + C, nf + 2).astype(np.int64)
        # stream order: (outer, inner) pairs, chunk-major when the plan loop-tiled the inner range
        q = P["chunk"]
        assert 1 <= q <= nRi and (q == nRi or (W_env() == 1 and P["split"] == 0))
        order = [(o, i) for c0 in range(0, nRi, q) for o in range(nRo) for i in range(c0, min(nRi, c0 + q))]
        oi = np.array(order, np.int64).reshape(-1, 2)
        oo, ii = oi[:, 0], oi[:, 1]
        np.testing.assert_array_equal(et[:nR], ro[oo, 0] * 8 + ri[ii, 0])
        assert (et[nR:] == 0).all() and (st[nR:, nf + 1] == -1).all()
        W = W_env()  # with the outer split every wave's first step loads
        starts = [0] + ([nRo * w // W * nRi for w in range(1, W)] if P["split"] == 1 else [])
        for j in range(nf):
            off = ro[oo, 4 + j] + ri[ii, 2 + j]
            assert (off % (C * 8) == 0).all()
            np.testing.assert_array_equal(st[:nR, j] & ~1, off)
            same = np.concatenate([[False], off[1:] == off[:-1]])
            same[[k for k in starts if k < nR]] = False
            np.testing.assert_array_equal((st[:nR, j] & 1) == 1, same)
        dw = (ro[oo, 1] & 0xFFFFFFFF) | (ri[ii, 1] & 0xFFFFFFFF)
        np.testing.assert_array_equal(st[:nR, nf] & 0xFFFFFFFF, dw)
        # a run's chunk end writes its bin (first chunk) or adds into it (-(bin + 2))
        end = (ii == np.minimum(nRi, (ii // q) * q + q) - 1)
        want = np.where(end, np.where(ii < q, ro[oo, 2], -(ro[oo, 2] + 2)), -1)
        np.testing.assert_array_equal(st[:nR, nf + 1], want)
    return [int(p[TE.F.index("chunk")]) for p in passes]


def W_env():
    return int(os.environ.get("FBN_JT_TW", "1"))


def test_step_records_alarm():
    _, (passes, tab, iv, geo) = _prog(ALARM)
    _check_steps(passes, tab, geo)


def test_step_records_munin_like(munin_fixture):
    _, (passes, tab, iv, geo) = _prog(munin_fixture["xml"])
    _check_steps(passes, tab, geo)


def test_step_records_loop_tiled(munin_fixture, monkeypatch):
    """FBN_JT_TILING = 1 (opt-in loop tiling of the inner range): chunk-major step order, a run's
    first chunk writes its bin and later chunks add into it; the emulated program still matches the
    reference's own Munin-like labels / marginals."""
    from conftest import read_ref_marg
    monkeypatch.setenv("FBN_JT_TILING", "1")
    jt, (passes, tab, iv, geo) = _prog(munin_fixture["xml"])
    chunks = _check_steps(passes, tab, geo)
    nri = [int(p[TE.F.index("nRi")]) for p in passes]
    assert sum(c < n for c, n in zip(chunks, nri)) > 50
    o = O.OracleJT(munin_fixture["xml"])
    ev, _ = O.load_libsvm(munin_fixture["libsvm"], o.n)
    rlab, rmarg, _, _ = read_ref_marg(munin_fixture["marg"], o.dims)
    lab, marg = TE.run((passes, tab, iv, geo), ev[:2], jt.info["sum_dom"])
    np.testing.assert_array_equal(lab, rlab[:2])
    np.testing.assert_allclose(marg, rmarg[:2], rtol=1e-9, atol=1e-300)


def test_step_records_four_wave_split(munin_fixture, monkeypatch):
    """FBN_JT_TW = 4 (four waves per case group): split passes, reuse bits cleared at every wave's
    first step."""
    monkeypatch.setenv("FBN_JT_TW", "4")
    _, (passes, tab, iv, geo) = _prog(munin_fixture["xml"])
    assert any(int(p[TE.F.index("split")]) == 1 for p in passes)
    _check_steps(passes, tab, geo)


def test_munin_like_extra_cases_vs_reference(munin_fixture):
    """The tiled program on one reference case per evidence level (0 / 52 / 208 / 520 observed)."""
    from conftest import read_ref_marg
    jt, prog = _prog(munin_fixture["xml"])
    o = O.OracleJT(munin_fixture["xml"])
    ev, _ = O.load_libsvm(munin_fixture["extra_libsvm"], o.n)
    rlab, rmarg, _, _ = read_ref_marg(munin_fixture["extra_marg"], o.dims)
    pick = [0, 16, 32, 48]
    lab, marg = TE.run(prog, ev[pick], jt.info["sum_dom"])
    np.testing.assert_array_equal(lab, rlab[pick])
    np.testing.assert_allclose(marg, rmarg[pick], rtol=1e-9, atol=1e-300)


def test_synth_nets_emulated_vs_reference(synth_nets):
    """The tiled program of a network with state counts up to 21 (plan limit was 8) and of one with
    a 12-variable clique (evidence on every clique variable, kernel loads past the 10th in a loop),
    emulated on the host, against the reference's own labels and marginals (tests/golden/synth_nets)."""
    for name, pick in (("bigdom", [0, 17, 40]), ("wide", list(range(0, 64, 5)))):
        fx = synth_nets[name]
        jt, prog = _prog(fx["xml"])
        lab, marg = TE.run(prog, fx["ev"][pick], jt.info["sum_dom"])
        np.testing.assert_array_equal(lab, fx["labels"][pick])
        np.testing.assert_allclose(marg, fx["marg"][pick], rtol=1e-9, atol=1e-300)
    assert max(synth_nets["bigdom"]["dims"]) == 21
