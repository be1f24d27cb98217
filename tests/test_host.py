"""Product host code without a GPU: the C-ABI library, loaders and the junction-tree plan builder."""
import ctypes
import os
import re

import numpy as np
import pytest
from conftest import GOLD, REPO, read_ci_fixture, read_pt_file, read_ref_marg, fnv1a

import fastbn_amd as F
import oracle as O


def header_symbols():
    txt = open(os.path.join(REPO, "include", "fastbn.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fbn_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(F.api.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 35
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python binding declares every one of them
    assert set(syms) - {"fbn_last_error"} <= set(F.api._SIGS)


def test_xmlbif_loader(alarm_paths):
    net = F.Network(alarm_paths["xml"])
    o = O.OracleJT(alarm_paths["xml"])
    assert net.num_nodes == 37
    np.testing.assert_array_equal(net.dims, o.dims)
    assert net.name(0) == "HISTORY" and net.name(36) == "BP"


def test_host_only_plan_matches_reference_dump(alarm_paths, tmp_path):
    net = F.Network(alarm_paths["xml"])
    jt = F.JunctionTree(net, device=-1)
    jt.dump_plan(str(tmp_path / "p"), str(tmp_path / "i"))
    assert open(tmp_path / "p").read() == open(os.path.join(GOLD, "alarm_1k.plan")).read()
    assert open(tmp_path / "i").read() == open(os.path.join(GOLD, "alarm_1k.init")).read()
    info = jt.info
    assert info["num_cliques"] == 27 and info["num_separators"] == 26 and info["num_levels"] == 15
    assert info["clique_entries"] == 1110 and info["separator_entries"] == 265
    assert info["algorithmic_bytes_per_case"] == 22877
    with pytest.raises(F.FastBNError, match="host-only"):
        jt.infer(np.full((1, 37), -1, np.int8))


def _counts_from_xmlbif(path):
    """(dims, parents in GIVEN order, counts [value][parent configs over ascending parents]) from the
    XMLBIF TABLE text alone (int(p * 10000), node-major, GIVEN order last fastest): an independent
    restatement of the count maps the reference's parser builds (src/XMLBIFParser.cpp:73-179)."""
    from fastbn_amd import synth
    import xml.etree.ElementTree as ET
    names, dims, parents, _ = synth.read_xmlbif(path)
    idx = {n: i for i, n in enumerate(names)}
    counts = [None] * len(names)
    for p in ET.parse(path).getroot().find("NETWORK").findall("PROBABILITY"):
        v = idx[p.find("FOR").text.strip()]
        given = [idx[g.text.strip()] for g in p.findall("GIVEN")]
        vals = [int(float(t) * 10000) for t in p.find("TABLE").text.strip().split(" ")]
        c = np.array(vals, np.int64).reshape([dims[v]] + [dims[g] for g in given])
        asc = sorted(given)
        c = np.transpose(c, [0] + [1 + given.index(q) for q in asc])  # parents to ascending order
        counts[v] = c.reshape(dims[v], -1)
    return names, dims, parents, counts


def test_network_from_counts_equals_xmlbif_path(alarm_paths, tmp_path):
    """fbn_network_create (a network handed over in memory, the reference's JunctionTree(Network*)
    binding) built from ALARM's count maps: the same node counts, the same plan and initial
    potentials as the XMLBIF path, byte for byte (the reference's own dump)."""
    names, dims, parents, counts = _counts_from_xmlbif(alarm_paths["xml"])
    net = F.Network.from_counts(dims, parents, counts, names)
    ref = F.Network(alarm_paths["xml"])
    np.testing.assert_array_equal(net.dims, ref.dims)
    for v in range(ref.num_nodes):
        pa, ca = net.node_counts(v)
        pb, cb = ref.node_counts(v)
        np.testing.assert_array_equal(pa, pb)
        np.testing.assert_array_equal(ca, cb)
    assert net.name(36) == "BP"
    jt = F.JunctionTree(net, device=-1)
    jt.dump_plan(str(tmp_path / "p"), str(tmp_path / "i"))
    assert open(tmp_path / "p").read() == open(os.path.join(GOLD, "alarm_1k.plan")).read()
    assert open(tmp_path / "i").read() == open(os.path.join(GOLD, "alarm_1k.init")).read()
    # bad inputs are reported, not fatal
    with pytest.raises(F.FastBNError, match="cycle"):
        F.Network.from_counts([2, 2], [[1], [0]], [np.ones((2, 2)), np.ones((2, 2))])
    with pytest.raises(F.FastBNError, match="bad parent"):
        F.Network.from_counts([2], [[3]], [np.ones((2, 2))])


def test_synthetic_network_plan_matches_oracle(tmp_path):
    from fastbn_amd import synth
    p = str(tmp_path / "syn.xml")
    synth.random_network(120, seed=7, window=8, path=p)
    jt = F.JunctionTree(F.Network(p), device=-1)
    o = O.OracleJT(p)
    jt.dump_plan(str(tmp_path / "a"), str(tmp_path / "b"))
    o.dump_plan(str(tmp_path / "c"), str(tmp_path / "d"))
    assert open(tmp_path / "a").read() == open(tmp_path / "c").read()
    assert open(tmp_path / "b").read() == open(tmp_path / "d").read()


def test_loaders_match_oracle_and_reference(alarm_paths):
    ds = F.Dataset(alarm_paths["csv"])
    od = O.OracleDataset(csv=alarm_paths["csv"])
    np.testing.assert_array_equal(ds.dims, od.dims)
    np.testing.assert_array_equal(ds.columns, od.columns)
    dims, colhash, _ = read_ci_fixture(os.path.join(GOLD, "alarm_s5000.ci.gz"))
    assert ds.dims.tolist() == dims
    assert all(fnv1a(ds.columns[v]) == h for v, h in colhash.items())
    assert ds.names[0] == "HISTORY"
    for key in ("test", "rand"):
        ev, lab = F.load_libsvm(alarm_paths[key], 37)
        oev, olab = O.load_libsvm(alarm_paths[key], 37)
        np.testing.assert_array_equal(ev, oev)
        np.testing.assert_array_equal(lab, olab)


def test_libsvm_unterminated_last_line_is_skipped(tmp_path):
    p = tmp_path / "t.libsvm"
    p.write_text("1 3:1 \n0 4:0")  # reference getline/eof loop never reads the last line
    ev, lab = F.load_libsvm(str(p), 37)
    assert ev.shape == (1, 37) and lab.tolist() == [1] and ev[0, 3] == 1


def test_score_matches_reference_mse(alarm_paths):
    """fbn_jt_score on the reference's own marginals reproduces its MSE/HD sums exactly."""
    net = F.Network(alarm_paths["xml"])
    jt = F.JunctionTree(net, device=-1)
    _, rmarg, mse_ref, hd_ref = read_ref_marg(os.path.join(GOLD, "alarm_1k.marg.gz"), net.dims)
    gold = read_pt_file(alarm_paths["pt"], net.dims, rmarg.shape[0])
    mse, hd = jt.score(rmarg, gold)
    assert mse == mse_ref and hd == hd_ref


def test_errors_are_reported_not_fatal(tmp_path):
    with pytest.raises(F.FastBNError, match="cannot open"):
        F.Network(str(tmp_path / "missing.xml"))
    bad = tmp_path / "bad.xml"
    bad.write_text("<BIF><NETWORK><VARIABLE><NAME>A</NAME><TYPE>discrete</TYPE><VALUE>x</VALUE>"
                   "<VALUE>y</VALUE></VARIABLE><PROBABILITY><FOR>A</FOR><TABLE>0.5 0.2 0.3 </TABLE>"
                   "</PROBABILITY></NETWORK></BIF>")
    with pytest.raises(F.FastBNError, match="too long"):
        F.Network(str(bad))
    with pytest.raises(F.FastBNError, match="cannot open"):
        F.Dataset(str(tmp_path / "missing.csv"))


# ---------------------------------------------------------------- PC orientation + SHD (host side)
def test_shd_matches_reference_fixture(alarm_paths):
    """fbn_shd_bif vs the reference's own BNSLComparison::GetSHD on 40 seeded learned graphs."""
    import json
    cases = json.load(open(os.path.join(GOLD, "alarm_shd.json")))
    bif = os.path.join(GOLD, "alarm", "alarm.bif")
    for c in cases:
        assert F.shd_bif(bif, 37, [tuple(e) for e in c["edges"]]) == c["shd"]


def test_orientation_alarm_known_answer():
    """PC-stable on alarm_s5000 (oracle skeleton): orientation == restatement, SHD == 5."""
    import oracle as O
    import orient
    od = O.OracleDataset(csv=os.path.join(GOLD, "alarm", "alarm_s5000.txt"))
    r = od.pc_stable(0.05, 1000, 1)
    res = F.orient_skeleton(37, r["edges"], r["sepset"])
    assert res.oriented == orient.orient(37, r["edges"], {k: tuple(v) for k, v in r["sepset"].items()})
    assert res.GetSHD(os.path.join(GOLD, "alarm", "alarm.bif")) == 5


def test_orientation_random_skeletons():
    """Random skeletons and sepsets (cycles, conflicting v-structures, Rule 3's position indexing);
    the dense trials give nodes more neighbours / parents than the node sets hold inline (6)."""
    import random
    import orient
    rng = random.Random(7)
    for trial in range(80):
        n = rng.randint(4, 14) if trial < 60 else rng.randint(12, 16)
        pairs = [(a, b) for a in range(n) for b in range(a + 1, n)]
        edges = [p for p in pairs if rng.random() < (0.35 if trial < 60 else 0.75)]
        sep = {}
        for p in pairs:
            if p not in edges:
                others = [v for v in range(n) if v not in p]
                sep[p] = tuple(sorted(rng.sample(others, rng.randint(0, min(3, len(others))))))
        res = F.orient_skeleton(n, edges, sep)
        assert res.oriented == orient.orient(n, edges, sep), trial


def test_orientation_larger_sparse_skeletons():
    """Sparse skeletons of 150-300 nodes (degree ~2-6, many v-structures, long Meek-rule sweeps):
    the indexed vec_edges (tombstoned slots, hashed first occurrence, positional sweeps) gives the
    restatement's edge list, order included."""
    import random
    import orient
    rng = random.Random(11)
    for trial in range(4):
        n = rng.randint(150, 300)
        edges = sorted({(min(a, b), max(a, b)) for a in range(n) for b in rng.sample(range(n), 2) if a != b})
        present = set(edges)
        sep = {}
        for a in range(n):
            for b in range(a + 1, min(n, a + 12)):  # sepsets of nearby absent pairs; others empty
                if (a, b) not in present:
                    others = [v for v in range(n) if v not in (a, b)]
                    sep[(a, b)] = tuple(sorted(rng.sample(others, rng.randint(0, 2))))
        res = F.orient_skeleton(n, edges, sep)
        assert res.oriented == orient.orient(n, edges, sep), trial


def _tree_from_dump(path):
    """parent clique of every clique from a plan dump ('c id ... | up s | down ...', 's id ... | up P | down C')."""
    sep_parent, clique_up = {}, {}
    for ln in open(path).read().split("\n"):
        if ln.startswith("s "):
            sid = int(ln.split()[1])
            sep_parent[sid] = int(ln.split("| up")[1].split("|")[0])
        elif ln.startswith("c "):
            cid = int(ln.split()[1])
            up = ln.split("| up")[1].split("|")[0].split()
            clique_up[cid] = int(up[0]) if up else -1
    return {c: (sep_parent[s] if s in sep_parent else -1) for c, s in clique_up.items()}


@pytest.mark.parametrize("net", ["alarm", "synth200", "munin_like"])
def test_streamed_schedule_respects_tree_dependencies(tmp_path, net):
    """Variant 4's block schedule (subtrees per wave in parallel, the top on one wave): every clique
    once per phase; Collect children before parents, Distribute parents before children, across
    the barrier-separated segments; subtrees never straddle waves."""
    from fastbn_amd import synth
    if net == "alarm":
        xml = os.path.join(GOLD, "alarm", "alarm.xml")
    else:
        xml = str(tmp_path / f"{net}.xml")
        if net == "synth200":
            synth.random_network(200, seed=11, window=10, path=xml)
        else:
            synth.random_network(1041, seed=1041, window=12, path=xml, name="munin_like")
    jt = F.JunctionTree(F.Network(xml), device=-1)
    assert jt.info["streamed_eligible"] == 1
    W = jt.info["streamed_waves"]
    order, sched = jt.stream_schedule()
    assert len(sched) == 2 * W + 3 and sched[-1] == len(order) == 2 * jt.info["num_cliques"]
    jt.dump_plan(str(tmp_path / "p"), str(tmp_path / "i"))
    parent = _tree_from_dump(str(tmp_path / "p"))
    nc = jt.info["num_cliques"]
    seg = [order[sched[i]:sched[i + 1]].tolist() for i in range(2 * W + 2)]
    col_w, col_top, dis_top, dis_w = seg[:W], seg[W], seg[W + 1], seg[W + 2:]
    assert sorted(sum(col_w, []) + col_top) == list(range(nc))
    assert sorted(sum(dis_w, []) + dis_top) == list(range(nc))
    assert sorted(col_top) == sorted(dis_top)
    owner = {c: w for w in range(W) for c in col_w[w]}
    assert owner == {c: w for w in range(W) for c in dis_w[w]}
    for c, w in owner.items():  # a subtree clique's parent: same wave or the top
        assert parent[c] == -1 or parent[c] in col_top or owner.get(parent[c]) == w
    # Collect: within a wave segment children first; the top runs after every wave segment
    for w in range(W):
        pos = {c: i for i, c in enumerate(col_w[w])}
        for c in col_w[w]:
            if parent[c] in pos:
                assert pos[parent[c]] > pos[c]
    pos = {c: i for i, c in enumerate(col_top)}
    for c in col_top:
        if parent[c] in pos:
            assert pos[parent[c]] > pos[c]
    # Distribute: the top first (parents first), then each wave's subtrees parents first
    pos = {c: i for i, c in enumerate(dis_top)}
    for c in dis_top:
        if parent[c] != -1:
            assert parent[c] in pos and pos[parent[c]] < pos[c]
    for w in range(W):
        pos = {c: i for i, c in enumerate(dis_w[w])}
        for c in dis_w[w]:
            if parent[c] in pos:
                assert pos[parent[c]] < pos[c]
    assert 0.5 < jt.info["streamed_split_efficiency"] <= 1.0 or W == 1


# ------------------------------------------------------------- native generators and text loaders
def test_native_generators_match_numpy(alarm_paths, tmp_path):
    """fbn_synth_forward_sample / fbn_synth_evidence draw exactly numpy's PCG64(seed) stream
    (SeedSequence, XSL-RR, 53-bit doubles, jump-ahead per thread): bit-identical to synth.py."""
    import fastbn_amd as F
    from fastbn_amd import synth
    net, py = F.Network(alarm_paths["xml"]), synth.read_xmlbif(alarm_paths["xml"])
    for seed in (0, 1, 1000, 20250131, 2 ** 40 + 7):
        np.testing.assert_array_equal(net.forward_sample(3001, seed), synth.forward_sample(py, 3001, seed))
    for n, k in ((1, 7), (513, 7), (20000, 7), (300, 0), (50, 36), (50, 40)):
        np.testing.assert_array_equal(net.evidence_cases(n, k, 20250131), synth.evidence_cases(py, n, k, 20250131))
    p = str(tmp_path / "syn.xml")
    synth.random_network(300, seed=5, window=12, path=p)
    np.testing.assert_array_equal(F.Network(p).evidence_cases(4097, 60, 9), synth.evidence_cases(synth.read_xmlbif(p), 4097, 60, 9))


def test_csv_writer_and_streaming_loader(tmp_path, monkeypatch):
    """fbn_write_csv -> fbn_dataset_load_csv (block-streamed, threaded): codes in first-appearance
    order per column (src/Dataset.cpp:334-342) across block and thread boundaries."""
    import fastbn_amd as F
    rng = np.random.default_rng(3)
    cols = rng.integers(0, 4, (7, 50001)).astype(np.uint8)
    cols[2] = 3 - cols[2] // 2  # codes whose first appearance is not 0, 1, ...
    cols[5] = 0  # a constant column
    p = str(tmp_path / "d.csv")
    F.write_csv(p, cols)
    for threads in ("1", "3", "8"):
        monkeypatch.setenv("OMP_NUM_THREADS", threads)
        ds = F.Dataset(p)
        assert ds.names == [f"X{v}" for v in range(7)]
        for v in range(7):
            vals, first = np.unique(cols[v], return_index=True)
            m = np.zeros(256, np.uint8)
            m[vals[np.argsort(first)]] = np.arange(len(vals))
            np.testing.assert_array_equal(ds.columns[v], m[cols[v]])
            assert ds.dims[v] == len(vals)


def test_libsvm_writer_and_streaming_loader(alarm_paths, tmp_path, monkeypatch):
    """fbn_write_libsvm -> fbn_evidence_load_libsvm round trip (labels, -1 for unobserved), and
    the reference's loader quirk: an unterminated last line is not read (src/Dataset.cpp:162-262)."""
    import fastbn_amd as F
    net = F.Network(alarm_paths["xml"])
    ev = net.evidence_cases(20001, 7, 4)
    lab = (np.arange(20001) % 3).astype(np.int32)
    p = str(tmp_path / "e.libsvm")
    F.write_libsvm(p, ev, lab)
    for threads in ("1", "5"):
        monkeypatch.setenv("OMP_NUM_THREADS", threads)
        e2, l2 = F.load_libsvm(p, 37)
        np.testing.assert_array_equal(e2, ev)
        np.testing.assert_array_equal(l2, lab)
    with open(p, "ab") as f:
        f.write(b"1 3:1")  # no newline: skipped like the reference's getline/eof loop
    e3, _ = F.load_libsvm(p, 37)
    assert e3.shape[0] == 20001
    # the shipped test set through the new loader = the oracle's loader
    e4, l4 = F.load_libsvm(alarm_paths["test"], 37)
    import oracle as O
    oe, ol = O.load_libsvm(alarm_paths["test"], 37)
    np.testing.assert_array_equal(e4, oe)
    np.testing.assert_array_equal(l4, ol)


def test_host_threads_under_tsan(alarm_paths, tmp_path):
    """SURVEY §5 race detection: the threaded host code (forward sampling, evidence generation, the
    chunked CSV / LIBSVM writers and the block-parallel parsers) built with ThreadSanitizer from its
    sources (g++ -fsanitize=thread, no HIP) and round-tripped on ALARM; any report fails the run."""
    import shutil
    import subprocess
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    csrc = os.path.join(REPO, "fastbn_amd", "csrc")
    exe = str(tmp_path / "host_tsan")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-I" + os.path.join(REPO, "include"),
                    os.path.join(csrc, "io.cpp"), os.path.join(csrc, "synth.cpp"),
                    os.path.join(REPO, "tests", "tsan", "host_tsan.cpp"), "-o", exe], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([exe, alarm_paths["xml"], str(tmp_path)], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "host_tsan ok" in r.stdout
