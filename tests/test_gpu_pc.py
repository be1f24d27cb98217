"""CI-test kernel and PC-stable driver vs the reference's counts and the oracle."""
import os

import numpy as np
import pytest
from conftest import GOLD, read_ci_fixture

import fastbn_amd as F
import oracle as O

pytestmark = pytest.mark.gpu

# G^2 = the reference's terms summed in its order (one running sum, src/IndependenceTest.cpp:94-138)
# with exact integer counts: the only difference left is the last bit of a term's log (the device
# log vs the host libm's std::log, which itself is not correctly rounded) -> a few ulp
# of the largest term (terms have both signs)
G2_TOL = 1e-12


@pytest.fixture(scope="module")
def alarm_ds(alarm_paths):
    return F.Dataset(alarm_paths["csv"])


@pytest.fixture(scope="module")
def ci(alarm_ds):
    return F.IndependenceTest(alarm_ds, 0.05, device=0)


def test_counts_bit_exact_vs_reference(ci):
    _, _, tests = read_ci_fixture(os.path.join(GOLD, "alarm_s5000.ci.gz"))
    for x, y, z, counts in tests:
        np.testing.assert_array_equal(ci.counts(x, y, z), counts)


def test_g2_df_p_vs_oracle(ci, alarm_paths):
    od = O.OracleDataset(csv=alarm_paths["csv"])
    _, _, tests = read_ci_fixture(os.path.join(GOLD, "alarm_s5000.ci.gz"))
    by_d = {}
    for x, y, z, _ in tests:
        by_d.setdefault(len(z), []).append([x, y] + z)
    for d, items in by_d.items():
        g2, df, p, ind = ci.run(np.array(items, np.int32), d)
        for k, it in enumerate(items):
            r = od.ci_test(it[0], it[1], it[2:])
            assert df[k] == r["df"]
            # the reference's running sum; only log's last bit can differ (glibc vs device)
            assert abs(g2[k] - r["g2"]) <= G2_TOL * max(1.0, abs(r["g2"]))  # north star: 1e-6 rel
            assert abs(p[k] - r["p_value"]) <= 1e-12  # p: parity unpinned (pchisq absent)
            assert ind[k] == r["is_independent"]


@pytest.mark.parametrize("gs,host", [(1, False), (1, True), (4, False)])
def test_pc_stable_alarm5000(alarm_ds, alarm_paths, gs, host, monkeypatch):
    """gs 1: the device-resident search (pc_small.hip, the default for <= 64 variables) and the
    host-driven level loop (FBN_PC_NO_SMALL); gs 4: grouped tests (host-driven)."""
    od = O.OracleDataset(csv=alarm_paths["csv"])
    ref = od.pc_stable(0.05, 1000, gs)
    if host:
        monkeypatch.setenv("FBN_PC_NO_SMALL", "1")
    pc = F.PCStable(0.05, 1000).StructLearnCompData(alarm_ds, group_size=gs)
    assert pc.tests_per_level.tolist() == ref["tests_per_level"]
    assert pc.edges == ref["edges"]
    assert pc.sepset == ref["sepset"]
    if gs == 1:
        assert pc.num_ci_test == 5206 and len(pc.edges) == 44
        # orientation (host) on the device skeleton: restatement edge for edge, SHD known answer
        import orient
        assert pc.oriented == orient.orient(37, pc.edges, pc.sepset)
        assert pc.GetSHD(alarm_paths["bif"]) == 5


@pytest.mark.parametrize("alpha,device_l1", [(0.001, False), (0.2, False), (0.2, True), (0.0, True)])
def test_pc_stable_alarm5000_other_alphas(alarm_ds, alarm_paths, alpha, device_l1, monkeypatch):
    """Decisions at other significance levels (depth 3): the decision band (ci_chisq.h
    fbn_chisq_band) is built per alpha (none at alpha 0: p evaluated for every test); device_l1
    forces the device-resident level-1 search.  Counts, skeleton and sepsets equal the
    restatement's."""
    od = O.OracleDataset(csv=alarm_paths["csv"])
    ref = od.pc_stable(alpha, 3, 1)
    monkeypatch.setenv("FBN_PC_NO_SMALL", "1")  # the host-driven level loop (pc_small: test_gpu_pc_small.py)
    if device_l1:
        monkeypatch.setenv("FBN_PC_FULLSPEC", "0")
    pc = F.PCStable(alpha, 3).StructLearnCompData(alarm_ds)
    assert pc.tests_per_level.tolist() == ref["tests_per_level"]
    assert pc.edges == ref["edges"]
    assert pc.sepset == ref["sepset"]


@pytest.mark.parametrize("fullspec", [True, False])
def test_level1_generators_agree(alarm_ds, alarm_paths, fullspec, monkeypatch):
    """Level-1 candidate generation: the single-pass writer (both sides of every edge in one round
    under full speculation, one slice per round otherwise) and the general per-test loop
    (FBN_PC_GEN_GENERAL) launch the same tests and give the restatement's result."""
    od = O.OracleDataset(csv=alarm_paths["csv"])
    ref = od.pc_stable(0.05, 1000, 1)
    monkeypatch.setenv("FBN_PC_NO_SMALL", "1")  # the host-driven level loop
    monkeypatch.setenv("FBN_PC_HOST_L1", "1")  # level 1 through the host rounds
    if not fullspec:
        monkeypatch.setenv("FBN_PC_FULLSPEC", "0")
    runs = []
    for general in (False, True):
        if general:
            monkeypatch.setenv("FBN_PC_GEN_GENERAL", "1")
        pc = F.PCStable(0.05, 1000).StructLearnCompData(alarm_ds)
        assert pc.tests_per_level.tolist() == ref["tests_per_level"]
        assert pc.edges == ref["edges"] and pc.sepset == ref["sepset"]
        runs.append(pc.launched_per_level.tolist())
    assert runs[0] == runs[1]


@pytest.mark.parametrize("gs,staged", [(1, False), (3, False), (1, True)])
def test_pc_stable_alarm5000_pipelined_rounds(alarm_ds, alarm_paths, gs, staged, monkeypatch):
    """The driver's multi-round path (no full speculation) with the level's edges in two halves
    alternating on the device (pc_driver.cpp), forced on ALARM: identical counts, skeleton and
    sepsets to the restatement, incl. grouped tests whose groups must not straddle rounds; staged:
    every round through the per-slot device buffers and DMA copies instead of zero-copy."""
    od = O.OracleDataset(csv=alarm_paths["csv"])
    ref = od.pc_stable(0.05, 1000, gs)
    monkeypatch.setenv("FBN_PC_NO_SMALL", "1")  # the host-driven level loop
    monkeypatch.setenv("FBN_PC_FULLSPEC", "0")
    monkeypatch.setenv("FBN_PC_PIPELINE_EDGES", "1")
    if staged:
        monkeypatch.setenv("FBN_CI_NO_ZEROCOPY", "1")
    pc = F.PCStable(0.05, 1000).StructLearnCompData(alarm_ds, group_size=gs)
    assert pc.tests_per_level.tolist() == ref["tests_per_level"]
    assert pc.edges == ref["edges"]
    assert pc.sepset == ref["sepset"]
    assert pc.launched_per_level.tolist() != [666, 5157, 1212, 128, 15]  # not the one-round schedule


@pytest.mark.parametrize("pairs", [True, False])
def test_pc_stable_alarm5000_bit_sliced_pair_tables(alarm_ds, alarm_paths, pairs, monkeypatch):
    """Levels 0-1 through the bit-sliced kernels (forced below their sample threshold): level 0
    records every pair's table, level 1 derives the last value of x, y and z from them
    (ci_bits_count_derived) -- identical counts, skeleton and sepsets to the restatement."""
    od = O.OracleDataset(csv=alarm_paths["csv"])
    ref = od.pc_stable(0.05, 1000, 1)
    monkeypatch.setenv("FBN_PC_NO_SMALL", "1")  # the host-driven level loop
    monkeypatch.setenv("FBN_CI_FORCE_BITS", "1")
    if not pairs:
        monkeypatch.setenv("FBN_CI_NO_PAIRS", "1")
    ci = F.IndependenceTest(alarm_ds)
    for _ in range(2):  # a second run on the same context re-records its own level 0
        pc = F.PCStable(0.05, 1000).StructLearnCompData(ci)
        assert pc.tests_per_level.tolist() == ref["tests_per_level"]
        assert pc.edges == ref["edges"]
        assert pc.sepset == ref["sepset"]
    # single tests after the run use full counting again (pair tables dropped at the end of the run)
    g2, df, p, ind = ci.run(np.array([[0, 1, 2], [5, 9, 30]], np.int32), 1)
    for k, (x, y, z) in enumerate([(0, 1, 2), (5, 9, 30)]):
        r = od.ci_test(x, y, [z])
        assert df[k] == r["df"] and ind[k] == r["is_independent"]


@pytest.mark.parametrize("rounds", ["default", "pipelined"])
def test_pc_stable_config5_like_vs_restatement(tmp_path, rounds, monkeypatch):
    """SURVEY config 5's generator at 150 variables x 50k samples, levels 0-5: every level-0/1
    test through the bit-sliced kernels (derived last values, recorded pair tables); "pipelined"
    forces multi-round levels in two halves -- identical test counts, skeleton and sepsets to the
    restatement."""
    if rounds == "pipelined":
        monkeypatch.setenv("FBN_PC_FULLSPEC", "0")
        monkeypatch.setenv("FBN_PC_PIPELINE_EDGES", "1")
    from fastbn_amd import synth
    path = str(tmp_path / "c5.xml")
    synth.random_network(150, seed=1000, window=50, parent_probs=(1, 1, 1), dom=(2, 4), path=path, k_min=0)
    cols = synth.forward_sample(synth.read_xmlbif(path), 50000, seed=1000)
    dims = (cols.max(axis=1).astype(np.int32) + 1)
    ref = O.OracleDataset(columns=cols, dims=dims).pc_stable(0.05, 6, 1)
    pc = F.PCStable(0.05, 6).StructLearnCompData(F.Dataset(columns=cols, dims=dims))
    assert pc.tests_per_level.tolist() == ref["tests_per_level"]
    assert pc.edges == ref["edges"]
    assert pc.sepset == ref["sepset"]


def test_pc_stable_synthetic_and_ragged_samples(tmp_path):
    from fastbn_amd import synth
    p = str(tmp_path / "syn.xml")
    synth.random_network(40, seed=3, window=6, path=p)
    cols = synth.forward_sample(synth.read_xmlbif(p), 4999, seed=4)  # N % 4 != 0 -> scalar path
    dims = cols.max(axis=1).astype(np.int32) + 1
    ds = F.Dataset(columns=cols, dims=dims)
    od = O.OracleDataset(columns=cols, dims=dims)
    ref = od.pc_stable(0.05, 1000, 1)
    pc = F.PCStable(0.05, 1000).StructLearnCompData(ds)
    assert pc.tests_per_level.tolist() == ref["tests_per_level"]
    assert pc.edges == ref["edges"] and pc.sepset == ref["sepset"]
    import orient
    assert pc.oriented == orient.orient(40, pc.edges, pc.sepset)


def test_constant_column_df0(tmp_path):
    cols = np.zeros((3, 1000), np.uint8)
    cols[1] = np.arange(1000) % 3
    cols[2] = (np.arange(1000) // 7) % 2
    ds = F.Dataset(columns=cols, dims=np.array([1, 3, 2], np.int32))
    r = F.IndependenceTest(ds).IndependenceResult(0, 1, (2,))
    assert r["df"] == 0 and r["is_independent"] and r["p_value"] == 1.0


def test_large_contingency_table_global_fallback():
    """|Z| = 7 over 4-state variables: 4^7 * 16 cells (1 MiB) exceed LDS -> global-memory tables;
    counts, df, G^2 and p must still match the restatement."""
    rng = np.random.default_rng(5)
    cols = rng.integers(0, 4, size=(10, 3001), dtype=np.uint8)
    cols[1] = (cols[0] + rng.integers(0, 2, size=3001)) % 4  # some dependence
    dims = np.full(10, 4, np.int32)
    ds = F.Dataset(columns=cols, dims=dims)
    od = O.OracleDataset(columns=cols, dims=dims)
    ci = F.IndependenceTest(ds)
    items = np.array([[0, 1, 2, 3, 4, 5, 6, 7, 8], [2, 9, 0, 1, 3, 4, 5, 6, 7]], np.int32)
    g2, df, p, ind = ci.run(items, 7)
    for k, it in enumerate(items):
        r = od.ci_test(int(it[0]), int(it[1]), [int(v) for v in it[2:]])
        assert df[k] == r["df"] and bool(ind[k]) == r["is_independent"]
        assert abs(g2[k] - r["g2"]) <= G2_TOL * max(1.0, abs(r["g2"]))
        assert abs(p[k] - r["p_value"]) <= 1e-12
    np.testing.assert_array_equal(ci.counts(0, 1, tuple(range(2, 9))),
                                  od.ci_test(0, 1, list(range(2, 9)), counts=True)["counts"])


def test_decision_margin_log(alarm_ds, alarm_paths):
    """every run logs min |p - alpha| (p-values are parity-unpinned).  The device
    evaluates a superset of the reference's tests (speculation), so its minimum is <= the
    reference-order minimum; ALARM-5000 has no decision within 1e-9 of alpha."""
    od = O.OracleDataset(csv=alarm_paths["csv"])
    ref = od.pc_stable(0.05, 1000, 1, keep_log=True)
    ref_min = min(abs(t[6] - 0.05) for t in ref["log"] if t[5] != 0)
    pc = F.PCStable(0.05, 1000).StructLearnCompData(alarm_ds)
    assert pc.near_alpha == 0
    assert 1e-9 < pc.min_margin <= ref_min * (1 + 1e-9)
    # the ctx-level log over an explicit batch equals the minimum over the returned p-values
    ci = F.IndependenceTest(alarm_ds)
    items = np.array([[t[1], t[2]] + list(t[3]) for t in ref["log"] if len(t[3]) == 1], np.int32)
    ci.decision_margin(reset=True)
    _, _, p, _ = ci.run(items, 1)
    m, near = ci.decision_margin()
    assert m == np.min(np.abs(p - 0.05)) and near == 0


@pytest.mark.parametrize("ns", [1, 31, 32, 33, 5000, 100003])
def test_bit_sliced_marginal_tests_match_histogram_kernel(ns):
    """Tests with <= 1 conditioning variable go through the bit-sliced popcount kernel (ci_bits.hip)
    when every variable has <= 4 states; the byte-column histogram kernel (FBN_CI_NO_BITS) must give identical counts,
    df, G^2 and p, and both must match the oracle.  Ragged sample counts, constant columns and
    1..4-state variables."""
    rng = np.random.default_rng(ns)
    nv = 12
    dims = np.array([1, 2, 3, 4, 2, 3, 4, 4, 2, 3, 1, 4], np.int32)
    cols = np.stack([rng.integers(0, d, ns) for d in dims]).astype(np.uint8)
    cols[5] = (cols[4] + cols[5]) % 3  # some dependence
    items0 = np.array([[x, y] for x in range(nv) for y in range(x + 1, nv)], np.int32)
    items1 = np.array([[x, y, z] for x in range(nv) for y in range(x + 1, nv) for z in range(nv)
                       if z != x and z != y], np.int32)
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims), 0.05, device=0)
    od = O.OracleDataset(columns=cols, dims=dims)
    os.environ["FBN_CI_FORCE_BITS"] = "1"  # the bit-sliced path also below its sample threshold
    try:
        res = {d: (ci.run(items, d), ci.counts(1, 7, [6] if d else [])) for d, items in ((0, items0), (1, items1))}
    finally:
        del os.environ["FBN_CI_FORCE_BITS"]
    for d, items in ((0, items0), (1, items1)):
        (g2, df, p, ind), cnt = res[d]
        os.environ["FBN_CI_NO_BITS"] = "1"
        try:
            g2h, dfh, ph, indh = ci.run(items, d)
            cnth = ci.counts(1, 7, [6] if d else [])
        finally:
            del os.environ["FBN_CI_NO_BITS"]
        np.testing.assert_array_equal(cnt, cnth)
        np.testing.assert_array_equal(df, dfh)
        np.testing.assert_array_equal(g2, g2h)
        np.testing.assert_array_equal(p, ph)
        np.testing.assert_array_equal(ind, indh)
        for k in range(0, len(items), max(1, len(items) // 25)):
            it = [int(v) for v in items[k]]
            r = od.ci_test(it[0], it[1], it[2:])
            assert df[k] == r["df"] and ind[k] == r["is_independent"]
            assert abs(g2[k] - r["g2"]) <= G2_TOL * max(1.0, abs(r["g2"]))


@pytest.mark.parametrize("ns", [33, 5000, 100003])
def test_bit_sliced_conditional_tables_match_byte_columns(ns):
    """FBN_CI_BITSN: d >= 2 tests whose variables all have <= 4 states count from the bit-sliced
    store (z-configurations x cells of popcount(x_a & y_b & AND of z rows)).  Tables, df, G^2 and p
    must equal the byte-column histogram kernel's and the oracle's, for ragged sample counts,
    1..4-state variables and d = 2, 3."""
    rng = np.random.default_rng(ns + 7)
    nv = 9
    dims = np.array([2, 3, 4, 1, 4, 3, 2, 4, 3], np.int32)
    cols = np.stack([rng.integers(0, d, ns) for d in dims]).astype(np.uint8)
    cols[4] = (cols[2] + cols[1]) % 4
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims), 0.05, device=0)
    od = O.OracleDataset(columns=cols, dims=dims)
    os.environ["FBN_CI_FORCE_BITS"] = "1"
    try:
        ci.run(np.array([[0, 1]], np.int32), 0)  # builds the bit-sliced store
    finally:
        del os.environ["FBN_CI_FORCE_BITS"]
    items2 = np.array([[x, y, a, b] for x in range(nv) for y in range(x + 1, nv) for a in range(nv) for b in
                       range(a + 1, nv) if len({x, y, a, b}) == 4][::7], np.int32)
    items3 = np.array([[0, 4, 1, 2, 7], [2, 5, 0, 4, 8], [1, 7, 3, 6, 5], [4, 8, 2, 0, 1]], np.int32)
    for d, items in ((2, items2), (3, items3)):
        os.environ["FBN_CI_BITSN"] = "1"
        try:
            g2, df, p, ind = ci.run(items, d)
            cnt = ci.counts(int(items[0][0]), int(items[0][1]), [int(v) for v in items[0][2:]])
        finally:
            del os.environ["FBN_CI_BITSN"]
        g2h, dfh, ph, indh = ci.run(items, d)
        cnth = ci.counts(int(items[0][0]), int(items[0][1]), [int(v) for v in items[0][2:]])
        np.testing.assert_array_equal(cnt, cnth)
        np.testing.assert_array_equal(df, dfh)
        np.testing.assert_array_equal(g2, g2h)
        np.testing.assert_array_equal(p, ph)
        np.testing.assert_array_equal(ind, indh)
        for k in range(0, len(items), max(1, len(items) // 20)):
            it = [int(v) for v in items[k]]
            r = od.ci_test(it[0], it[1], it[2:])
            assert df[k] == r["df"] and ind[k] == r["is_independent"]
            assert abs(g2[k] - r["g2"]) <= G2_TOL * max(1.0, abs(r["g2"]))


@pytest.mark.parametrize("ns", [33, 5000, 100003])
def test_packed_columns_match_byte_columns(ns, monkeypatch):
    """Histogram-kernel batches whose variables all have <= 4 states read the columns packed 2 bits
    per sample (16 per word, the tail word's padding excluded): tables, df, G^2, p and decisions
    equal the byte-column kernel's (FBN_CI_NO_PACK2) and the oracle's, for ragged sample counts and
    d = 0..4; a batch with a 5-state variable keeps the byte columns."""
    rng = np.random.default_rng(ns + 11)
    dims = np.array([2, 3, 4, 1, 4, 3, 2, 4, 3, 5], np.int32)
    nv = len(dims)
    cols = np.stack([rng.integers(0, d, ns) for d in dims]).astype(np.uint8)
    cols[4] = (cols[2] + cols[1]) % 4
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims), 0.05, device=0)
    od = O.OracleDataset(columns=cols, dims=dims)
    monkeypatch.setenv("FBN_CI_PACK2", "1")  # the packed columns at every sample count
    batches = {
        0: np.array([[x, y] for x in range(9) for y in range(x + 1, 9)], np.int32),
        1: np.array([[0, 4, 2], [1, 2, 4], [5, 8, 7], [3, 6, 0]], np.int32),
        2: np.array([[x, y, a, b] for x in range(9) for y in range(x + 1, 9) for a in range(9) for b in
                     range(a + 1, 9) if len({x, y, a, b}) == 4][::11], np.int32),
        3: np.array([[0, 4, 1, 2, 7], [2, 5, 0, 4, 8], [1, 7, 3, 6, 5]], np.int32),
        4: np.array([[0, 4, 1, 2, 7, 8], [2, 5, 0, 4, 8, 6]], np.int32),
        5: np.array([[0, 9, 1, 2, 7, 8, 4]], np.int32),  # 5-state variable: byte columns
    }
    for d, items in batches.items():
        g2, df, p, ind = ci.run(items, d)
        cnt = ci.counts(int(items[0][0]), int(items[0][1]), [int(v) for v in items[0][2:]])
        os.environ["FBN_CI_NO_PACK2"] = "1"
        try:
            g2b, dfb, pb, indb = ci.run(items, d)
            cntb = ci.counts(int(items[0][0]), int(items[0][1]), [int(v) for v in items[0][2:]])
        finally:
            del os.environ["FBN_CI_NO_PACK2"]
        np.testing.assert_array_equal(cnt, cntb)
        np.testing.assert_array_equal(df, dfb)
        np.testing.assert_array_equal(g2, g2b)
        np.testing.assert_array_equal(p, pb)
        np.testing.assert_array_equal(ind, indb)
        for k in range(0, len(items), max(1, len(items) // 10)):
            it = [int(v) for v in items[k]]
            r = od.ci_test(it[0], it[1], it[2:])
            assert df[k] == r["df"] and ind[k] == r["is_independent"]
            assert abs(g2[k] - r["g2"]) <= G2_TOL * max(1.0, abs(r["g2"]))


def test_level0_batches_and_device_compaction_match_single_batch():
    """Level 0 of the complete graph in bounded batches (FBN_PC_L0CHUNK) with the kept pairs
    compacted on the device per batch: the same skeleton, sepsets and counts as one batch, on a
    400-variable x 20k synthetic dataset (79,800 pairs: the device-compaction path)."""
    from fastbn_amd import synth
    cols, dims = synth.config5_dataset(400, 20000)
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
    a = F.PCStable(0.05, 3).StructLearnCompData(ci)
    os.environ["FBN_PC_L0CHUNK"] = "9999"
    try:
        b = F.PCStable(0.05, 3).StructLearnCompData(ci)
    finally:
        del os.environ["FBN_PC_L0CHUNK"]
    assert a.edges == b.edges and a.sepset == b.sepset
    assert a.tests_per_level.tolist() == b.tests_per_level.tolist()
    assert a.oriented == b.oriented


def test_g2_within_1e12_every_alarm5000_test(ci, alarm_paths):
    """Every CI test the reference's PC-stable run executes on ALARM-5000 (5206 tests, levels 0-4,
    from the restatement's log): G^2 within 1e-12 of max(1, |G^2|) -- the reference's single running
    sum over z -> x -> y (src/IndependenceTest.cpp:94-138) of the same terms; only the last bit of a
    term's log can differ (device log vs glibc's; north star: 1e-6) -- df and decisions
    identical, p within 1e-12 (pchisq parity unpinned)."""
    od = O.OracleDataset(csv=alarm_paths["csv"])
    ref = od.pc_stable(0.05, 1000, 1, keep_log=True)
    by_d = {}
    for t in ref["log"]:
        by_d.setdefault(len(t[3]), []).append(t)
    assert sum(len(v) for v in by_d.values()) == 5206
    for d, log in by_d.items():
        items = np.array([[t[1], t[2]] + list(t[3]) for t in log], np.int32)
        g2, df, p, ind = ci.run(items, d)
        ref_g2 = np.array([t[4] for t in log])
        assert np.all(np.abs(g2 - ref_g2) <= G2_TOL * np.maximum(1.0, np.abs(ref_g2)))
        np.testing.assert_array_equal(df, np.array([t[5] for t in log]))
        np.testing.assert_array_equal(ind.astype(bool), np.array([t[7] for t in log], bool))
        assert np.max(np.abs(p - np.array([t[6] for t in log]))) <= 1e-12


def test_kernel_timing_switch(alarm_ds):
    """fbn_ci_set_kernel_timing: events off -> identical results, kernel times read 0; back on."""
    ci = F.IndependenceTest(alarm_ds)
    a = F.PCStable(0.05, 1000).StructLearnCompData(ci)
    assert a.kernel_s > 0
    ci.set_kernel_timing(False)
    b = F.PCStable(0.05, 1000).StructLearnCompData(ci)
    assert b.kernel_s == 0 and b.edges == a.edges and b.sepset == a.sepset
    assert b.tests_per_level.tolist() == a.tests_per_level.tolist()
    ci.run(np.array([[0, 1]], np.int32), 0)
    assert ci.last_kernel_ms() == 0
    ci.set_kernel_timing(True)
    ci.run(np.array([[0, 1]], np.int32), 0)
    assert ci.last_kernel_ms() > 0


def test_pc_stable_config5_full_size_vs_fixture():
    """BASELINE config 5 at full size (1000 variables x 100k samples, depth 6): the device
    skeleton vs the restatement's committed result (tests/golden/pc_c5.json, 801,354 tests):
    identical tests per level, edge list and sepsets (digests), on the regenerated dataset."""
    import hashlib
    import json
    from conftest import pc_digest
    from fastbn_amd import synth
    ref = json.load(open(os.path.join(GOLD, "pc_c5.json")))
    cols, dims = synth.config5_dataset()
    assert hashlib.sha256(np.ascontiguousarray(cols).tobytes()).hexdigest() == ref["columns_sha256"]
    assert dims.tolist() == ref["dims"]
    pc = F.PCStable(ref["alpha"], ref["depth"]).StructLearnCompData(F.Dataset(columns=cols, dims=dims))
    assert pc.tests_per_level.tolist() == ref["tests_per_level"]
    assert pc.num_ci_test == ref["num_ci_test"] == 801354
    assert len(pc.edges) == ref["num_edges"] and len(pc.sepset) == ref["num_sepsets"]
    assert pc_digest(pc.edges, pc.sepset) == {k: ref[k] for k in ("edges_sha256", "sepsets_sha256")}
    assert pc.near_alpha == 0


@pytest.mark.parametrize("ns", [4096, 5000, 100003])
def test_level2_derived_counting_matches_histogram(ns, monkeypatch):
    """d = 2 tests inside a PC run (level-0 pair tables recorded), every state count <= 4: the
    derived bit-sliced counting (ci_kernels.hip MODE 3: leading 4-way and 3-way cells by popcount,
    the rest by subtraction from the pair tables) gives the histogram kernel's tables exactly
    (FBN_CI_NO_DER2), hence the same df, G^2, p and decisions bit for bit, and the oracle's."""
    rng = np.random.default_rng(ns + 29)
    dims = np.array([2, 3, 4, 1, 4, 3, 2, 4, 3, 4, 2], np.int32)
    cols = np.stack([rng.integers(0, d, ns) for d in dims]).astype(np.uint8)
    cols[4] = (cols[2] + cols[1]) % 4
    cols[9] = (cols[7] * cols[0] + cols[5]) % 4
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims), 0.05, device=0)
    od = O.OracleDataset(columns=cols, dims=dims)
    nv = len(dims)
    items = np.array([[x, y, a, b] for x in range(nv) for y in range(x + 1, nv) for a in range(nv)
                      for b in range(a + 1, nv) if len({x, y, a, b}) == 4][::7], np.int32)
    cap = 256
    got = ci.production_counts(items, 2, cap)  # records level 0's pair tables first
    g2, df, p, ind = ci.run(items, 2)
    monkeypatch.setenv("FBN_CI_NO_DER2", "1")
    ref = ci.production_counts(items, 2, cap)
    g2b, dfb, pb, indb = ci.run(items, 2)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(df, dfb)
    np.testing.assert_array_equal(g2, g2b)
    np.testing.assert_array_equal(p, pb)
    np.testing.assert_array_equal(ind, indb)
    for k in range(0, len(items), max(1, len(items) // 12)):
        it = [int(v) for v in items[k]]
        r = od.ci_test(it[0], it[1], it[2:])
        assert df[k] == r["df"] and ind[k] == r["is_independent"]
        assert abs(g2[k] - r["g2"]) <= G2_TOL * max(1.0, abs(r["g2"]))


@pytest.mark.parametrize("nvars,ns", [(333, 20000), (1000, 100000)])
def test_level0_to_level1_on_device_matches_host_path(nvars, ns, monkeypatch):
    """Level 0 -> level 1 without the host round trip (the kept pairs become the level-1 edge list
    and CSR adjacency on the device, ci_kept_* kernels; the host builds its copies while level 1
    runs) against the host path (FBN_PC_HOST_L0L1=1): the same skeleton, sepsets, counted and
    launched tests and orientation; 333 variables (ballot tails: not a multiple of 64) and config 5."""
    from fastbn_amd import synth
    cols, dims = synth.config5_dataset(nvars, ns)
    # a fresh context: the first run must take the device hand-off (fbn_pc_path 3), not only warm runs
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
    a = F.PCStable(0.05, 6).StructLearnCompData(ci)
    assert a.path == 3
    monkeypatch.setenv("FBN_PC_HOST_L0L1", "1")
    b = F.PCStable(0.05, 6).StructLearnCompData(F.IndependenceTest(F.Dataset(columns=cols, dims=dims)))
    assert b.path == 0
    assert a.edges == b.edges and a.sepset == b.sepset
    assert a.tests_per_level.tolist() == b.tests_per_level.tolist()
    assert a.launched_per_level.tolist() == b.launched_per_level.tolist()
    assert a.oriented == b.oriented


def test_level1_information_screen_config5(monkeypatch):
    """The level-1 information screen (ci_bits.hip l1_plausible: a candidate z with I(X;Z) or I(Y;Z)
    below I(X;Y) - hi(df) / 2N is certainly dependent and not run) on config 5 at full size: the same
    counted tests, skeleton, sepsets and orientation as every candidate run (FBN_PC_NO_MISCREEN), both
    equal to the fixture; level 1 runs far fewer tests than it counts."""
    import json
    from conftest import GOLD, pc_digest
    from fastbn_amd import synth
    cols, dims = synth.config5_dataset(1000, 100000)
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
    a = F.PCStable(0.05, 6).StructLearnCompData(ci)
    monkeypatch.setenv("FBN_PC_NO_MISCREEN", "1")
    b = F.PCStable(0.05, 6).StructLearnCompData(ci)
    monkeypatch.delenv("FBN_PC_NO_MISCREEN")
    ref = json.load(open(os.path.join(GOLD, "pc_c5.json")))
    for r in (a, b):
        assert r.tests_per_level.tolist() == ref["tests_per_level"]
        assert pc_digest(r.edges, r.sepset) == {k: ref[k] for k in ("edges_sha256", "sepsets_sha256")}
    assert a.oriented == b.oriented
    la, lb = a.launched_per_level.tolist(), b.launched_per_level.tolist()
    assert la[1] < 0.5 * a.tests_per_level.tolist()[1] and lb[1] >= b.tests_per_level.tolist()[1]


@pytest.mark.parametrize("alpha", [0.001, 0.01, 0.2, 0.5])
def test_level1_information_screen_alphas_vs_oracle(alpha, monkeypatch):
    """The screen's threshold moves with alpha (the band's hi per df): on a 200-variable config-5-like
    dataset (20k samples: the device level-1 rounds run) the screened run equals the unscreened one
    and the restatement -- tests per level, skeleton, sepsets."""
    from fastbn_amd import synth
    cols, dims = synth.config5_dataset(200, 20000)
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
    a = F.PCStable(alpha, 6).StructLearnCompData(ci)
    monkeypatch.setenv("FBN_PC_NO_MISCREEN", "1")
    b = F.PCStable(alpha, 6).StructLearnCompData(F.IndependenceTest(F.Dataset(columns=cols, dims=dims)))
    monkeypatch.delenv("FBN_PC_NO_MISCREEN")
    o = O.OracleDataset(columns=cols, dims=dims).pc_stable(alpha, 6, 1)
    assert a.tests_per_level.tolist() == b.tests_per_level.tolist() == o["tests_per_level"]
    assert a.edges == b.edges == o["edges"] and a.sepset == b.sepset == o["sepset"]
    assert a.launched_per_level.tolist()[1] <= b.launched_per_level.tolist()[1]
