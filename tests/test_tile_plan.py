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
