"""Config 5 (1000 variables x 100k samples) pinned against the UNMODIFIED reference's counting at
full scale: tests/golden/pc_c5.ci.gz holds Counts2D / Counts3D::FillTable tables (src/CellTable.cpp,
compiled in place by oracle/Makefile into oracle/_ref/ref_dump) for a seeded sample of the tests a
config-5 run performs at every level 0-5, with the FNV-1a hash of every column the reference read
(tests/golden/make_golden_synth.py c5ci).  The device computes the same tests through the kernels a
PC run uses at each level (fbn_ci_debug_counts: level-0 Gram of the leading mask rows + pair tables,
derived level-1 counting from them, the 2-bit packed histogram kernel for levels 2-5): counts equal
the reference's exactly; df / G^2 / decisions equal the restatement's (G^2 within 1e-12 of max(1,
|G^2|), p parity-unpinned)."""
import os

import numpy as np
import pytest
from conftest import GOLD, fnv1a_columns, read_ci_fixture

import fastbn_amd as F
import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c5():
    from fastbn_amd import synth
    dims, colhash, tests = read_ci_fixture(os.path.join(GOLD, "pc_c5.ci.gz"))
    cols, gdims = synth.config5_dataset()
    assert gdims.tolist() == dims
    h = fnv1a_columns(cols)
    assert all(int(h[v]) == colhash[v] for v in range(len(dims)))  # the reference read these columns
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=gdims))
    return cols, gdims, ci, tests


def _by_level(tests):
    out = {}
    for x, y, z, counts in tests:
        out.setdefault(len(z), []).append((x, y, z, counts))
    return out


def test_fixture_covers_levels_0_to_5(c5):
    lv = _by_level(c5[3])
    assert sorted(lv) == [0, 1, 2, 3, 4, 5]


@pytest.mark.parametrize("d", [0, 1, 2, 3, 4, 5])
def test_production_counts_equal_reference(c5, d):
    _, dims, ci, tests = c5
    lv = _by_level(tests)[d]
    items = np.array([[x, y] + z for x, y, z, _ in lv], np.int32)
    cap = max(len(c) for *_, c in lv)
    got = ci.production_counts(items, d, cap)
    for k, (_, _, _, ref) in enumerate(lv):
        np.testing.assert_array_equal(got[k, :len(ref)], ref, err_msg=f"level {d} test {k}: {items[k].tolist()}")
    if d >= 2:  # also as part of a batch > 512 tests (the 256-thread instantiation config-5 levels use)
        reps = 513 // len(items) + 1
        big = ci.production_counts(np.tile(items, (reps, 1)), d, cap)
        np.testing.assert_array_equal(big[:len(items)], got)


@pytest.mark.parametrize("d", [0, 1, 2, 3, 4, 5])
def test_df_g2_decisions_vs_restatement(c5, d):
    cols, dims, ci, tests = c5
    od = O.OracleDataset(columns=cols, dims=dims)
    lv = _by_level(tests)[d]
    items = np.array([[x, y] + z for x, y, z, _ in lv], np.int32)
    g2, df, p, ind = ci.run(items, d)
    for k, it in enumerate(items):
        r = od.ci_test(int(it[0]), int(it[1]), [int(v) for v in it[2:]])
        assert df[k] == r["df"] and bool(ind[k]) == r["is_independent"]
        assert abs(g2[k] - r["g2"]) <= 1e-12 * max(1.0, abs(r["g2"]))
        assert abs(p[k] - r["p_value"]) <= 1e-12


def _config5_full_size(monkeypatch, env):
    import hashlib
    import json
    from conftest import pc_digest
    from fastbn_amd import synth
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ref = json.load(open(os.path.join(GOLD, "pc_c5.json")))
    cols, dims = synth.config5_dataset()
    assert hashlib.sha256(np.ascontiguousarray(cols).tobytes()).hexdigest() == ref["columns_sha256"]
    pc = F.PCStable(ref["alpha"], ref["depth"]).StructLearnCompData(F.Dataset(columns=cols, dims=dims))
    assert pc.tests_per_level.tolist() == ref["tests_per_level"]
    assert pc_digest(pc.edges, pc.sepset) == {k: ref[k] for k in ("edges_sha256", "sepsets_sha256")}


def test_config5_full_size_default_mfma_gram(monkeypatch):
    """Config 5 at full size on the default path (level 0's Gram on the hand-written FP4 MFMA
    kernel, no library GEMM): the restatement's tests per level, edges, sepsets."""
    _config5_full_size(monkeypatch, {})


def test_config5_full_size_popcount_gram(monkeypatch):
    """The same with level 0's Gram on the hand-written popcount kernel (FBN_CI_GRAM_NO_MFMA)."""
    _config5_full_size(monkeypatch, {"FBN_CI_GRAM_NO_MFMA": "1"})
