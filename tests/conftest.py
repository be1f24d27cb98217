"""Shared fixtures.  `-m "not gpu"` runs here (no GPU); `-m gpu` runs on an MI355X box."""
import gzip
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
ALARM = os.path.join(GOLD, "alarm")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def read_ref_marg(path, dims):
    """Parse a reference harness .marg(.gz) dump -> (labels, marginals [n][sum dom], mse_sum, hd_sum)."""
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        lines = f.read().split("\n")
    labels, rows, i, mse, hd = [], [], 0, None, None
    V = len(dims)
    while i < len(lines):
        ln = lines[i]
        if ln.startswith("case"):
            labels.append(int(ln.split()[3]))
            row = []
            for v in range(V):
                row += [float(x) for x in lines[i + 1 + v].split()]
            rows.append(row)
            i += 1 + V
        elif ln.startswith("mse_sum"):
            t = ln.split()
            mse, hd = float(t[1]), float(t[3])
            i += 1
        else:
            i += 1
    return np.array(labels, np.int32), np.array(rows), mse, hd


def read_pt_file(path, dims, ncases):
    """alarm_1k_pt -> golden [n][sum dom] with -1 in the first slot of evidence nodes."""
    SD = int(np.sum(dims))
    out = np.zeros((ncases, SD))
    with open(path) as f:
        lines = f.read().split("\n")
    k = 0
    for c in range(ncases):
        off = 0
        for v, d in enumerate(dims):
            ln = lines[k].rstrip()
            k += 1
            if not ln:
                out[c, off] = -1
            else:
                out[c, off:off + d] = [float(x) for x in ln.split(" ")[:d]]
            off += d
    return out


def read_ci_fixture(path):
    with gzip.open(path, "rt") as f:
        lines = f.read().strip().split("\n")
    dims = [int(x) for x in lines[1].split()[1:]]
    colhash = {}
    tests = []
    for ln in lines[2:]:
        t = ln.split()
        if t[0] == "colhash":
            colhash[int(t[1])] = int(t[2])
        elif t[0] == "test":
            x, y, d = int(t[1]), int(t[2]), int(t[3])
            z = [int(v) for v in t[4:4 + d]]
            colon = t.index(":")
            counts = np.array([int(v) for v in t[colon + 1:]], np.int32)
            tests.append((x, y, z, counts))
    return dims, colhash, tests


def gram_dataset(nvars, N, seed):
    """Seeded ragged-shape datasets of the level-0 Gram tests (test_gpu_gram_mfma.py and the
    reference fixture tests/golden/gram_ragged.ci.gz, make_golden_synth.py gram): state counts 2-4,
    mildly dependent columns (tables far from uniform), and a sample of pairs that includes the
    first / last rows of the 256-row Gram tiles."""
    rng = np.random.default_rng(seed)
    dims = rng.integers(2, 5, nvars).astype(np.int32)
    cols = np.empty((nvars, N), np.uint8)
    base = rng.integers(0, 4, N)
    for v in range(nvars):
        noise = rng.integers(0, dims[v], N)
        keep = rng.random(N) < 0.3
        cols[v] = np.where(keep, base % dims[v], noise)
    rng = np.random.default_rng(seed + 100)
    x = rng.integers(0, nvars - 1, 1500)
    y = np.minimum(nvars - 1, x + 1 + rng.integers(0, nvars, 1500))
    pairs = np.unique(np.stack([x, y], 1), axis=0)
    pairs = np.concatenate([pairs, [[0, 1], [0, nvars - 1], [nvars - 2, nvars - 1]]]).astype(np.int32)
    return cols, dims, pairs


def fnv1a_columns(cols):
    """FNV-1a 64 over every column's int values (ref_dump ci's colhash), vectorised across columns."""
    h = np.full(cols.shape[0], 1469598103934665603, np.uint64)
    prime = np.uint64(1099511628211)
    with np.errstate(over="ignore"):
        for k in range(cols.shape[1]):
            h ^= cols[:, k].astype(np.uint64)
            h *= prime
    return h


def read_ci_blocks(path):
    """Multi-block ci fixture (gram_ragged.ci.gz): {(nvars, N, seed): (dims, colhash, tests)}."""
    import tempfile
    with gzip.open(path, "rt") as f:
        text = f.read()
    out = {}
    for blk in text.split("shape ")[1:]:
        head, body = blk.split("\n", 1)
        key = tuple(int(v) for v in head.split())
        with tempfile.NamedTemporaryFile("wb", suffix=".gz") as tf:
            with gzip.open(tf.name, "wt") as g:
                g.write(body)
            out[key] = read_ci_fixture(tf.name)
    return out


GRAM_SHAPES = [(520, 30001, 1), (700, 20480, 2), (260, 100003, 3)]


def pc_digest(edges, sepset):
    """Digests of a PC-stable skeleton: the edge list in vec_edges order and the sepsets as
    (x, y, |Z|, Z...) records in ascending key order (int32), sha256 hex."""
    import hashlib
    e = np.asarray(edges, np.int32).reshape(-1, 2)
    rec = []
    for k in sorted(sepset):
        z = sorted(sepset[k])
        rec += [k[0], k[1], len(z)] + list(z)
    return {"edges_sha256": hashlib.sha256(e.tobytes()).hexdigest(),
            "sepsets_sha256": hashlib.sha256(np.asarray(rec, np.int32).tobytes()).hexdigest()}


def fnv1a(col):
    h = 1469598103934665603
    for v in col.tolist():
        h ^= v
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.fixture(scope="session")
def alarm_paths():
    return {k: os.path.join(ALARM, v) for k, v in {
        "xml": "alarm.xml", "bif": "alarm.bif", "test": "testing_alarm_1k_p20", "pt": "alarm_1k_pt",
        "csv": "alarm_s5000.txt", "rand": "rand_evidence.libsvm"}.items()}


def have_gpu():
    try:
        import fastbn_amd
        return fastbn_amd.device_count() > 0
    except Exception:
        return False


MUNIN = os.path.join(GOLD, "munin_like")


@pytest.fixture(scope="session")
def munin_fixture(tmp_path_factory):
    """BASELINE config 4 fixture (tests/golden/make_golden_synth.py): the seeded Munin-like XMLBIF,
    32 evidence cases and the reference's own labels / marginals / plan for them."""
    d = tmp_path_factory.mktemp("munin_like")
    xml = str(d / "munin_like.xml")
    with gzip.open(os.path.join(MUNIN, "munin_like.xml.gz"), "rb") as f, open(xml, "wb") as g:
        g.write(f.read())
    lib = str(d / "ev.libsvm")
    with gzip.open(os.path.join(MUNIN, "ev.libsvm.gz"), "rb") as f, open(lib, "wb") as g:
        g.write(f.read())
    plan = str(d / "ref.plan")
    with gzip.open(os.path.join(MUNIN, "ref.plan.gz"), "rb") as f, open(plan, "wb") as g:
        g.write(f.read())
    extra = str(d / "extra_ev.libsvm")
    with gzip.open(os.path.join(MUNIN, "extra_ev.libsvm.gz"), "rb") as f, open(extra, "wb") as g:
        g.write(f.read())
    return {"xml": xml, "libsvm": lib, "plan": plan, "marg": os.path.join(MUNIN, "ref.marg.gz"),
            # 64 more cases at 0 / 52 / 208 / 520 observed variables (make_golden_synth.py munin_extra)
            "extra_libsvm": extra, "extra_marg": os.path.join(MUNIN, "extra_ref.marg.gz")}


def parse_plan(path):
    """A plan dump (fbn_jt_plan_dump / the reference harness) -> cliques {id: (vars, up, down)},
    separators {id: (vars, up, down)}, root, levels."""
    C, S, root, levels = {}, {}, None, []
    for ln in open(path):
        t = ln.split()
        if t and t[0] in ("c", "s"):
            i, nv = int(t[1]), int(t[2])
            up = int(t[t.index("up") + 1])
            down = [int(v) for v in t[t.index("down") + 1:]]
            (C if t[0] == "c" else S)[i] = (tuple(int(v) for v in t[4:4 + nv]), up, down)
        elif t and t[0] == "root":
            root = int(t[1])
        elif t and t[0] == "level":
            levels.append([int(v) for v in t[3:]])
    return C, S, root, levels


# the reference's junction tree on the Munin-like network depends on heap addresses (Prim's ties
# between equal-weight separators are broken by the pointer order of a std::set<Separator*>,
# src/JunctionTreeStructure.cpp:231,264-277); ours breaks them by creation order.  Both are
# maximum-weight spanning trees over the same cliques; message order then differs on the tied
# branches, so the marginals agree to a few ulp, labels exactly.
MUNIN_REF_RTOL = 1e-12


# ---- seeded networks beyond ALARM / Munin-like: state counts up to 21 (the reference's own networks
# -- Hailfinder, Diabetes, Munin -- have such variables), a 12-variable clique, and symmetric CPTs
# whose query marginals tie.  Fixtures: tests/golden/make_golden_synth.py synth_nets (the reference's
# own labels and marginals, oracle/_ref/ref_dump jt).
SYNTH_NETS = os.path.join(GOLD, "synth_nets")
SYNTH_NET_SPECS = {
    "bigdom": dict(n_nodes=120, seed=21, window=6, parent_probs=(0.75, 0.25), dom=(2, 21)),
    "wide": dict(n_nodes=48, seed=11, window=12, parent_probs=(0.85, 0.15), dom=(2, 2), fan_in={14: 11, 30: 6}),
}
# evidence cases per fixture: (cases, observed variables, seed) blocks
SYNTH_NET_CASES = {"bigdom": [(16, 0, 5), (16, 24, 6), (16, 60, 7)],
                   "wide": [(24, 10, 8), (24, 30, 9), (16, 47, 10)],
                   "tie": [(32, 4, 11), (32, 8, 12)]}


def tie_network(path, n_sym=8, n_extra=40, seed=3):
    """Query X0 (binary, 0.5 / 0.5) with n_sym binary children whose CPTs are symmetric under
    swapping X0's values (P(c | X0 = 0) = (a, b), P(c | X0 = 1) = (b, a)), so X0's posterior ties
    exactly whenever as many observed children are 0 as 1 (and with none observed); plus n_extra
    seeded nodes hanging off the children (a larger tree).  Written as XMLBIF (node-major TABLE)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = 1 + n_sym + n_extra
    parents, tables = [[]], [[0.5, 0.5]]
    for i in range(1, 1 + n_sym):
        parents.append([0])
        tables.append([0.3, 0.7, 0.7, 0.3])  # node-major: [value][X0]
    for i in range(1 + n_sym, n):
        p = int(rng.integers(1, i))
        parents.append([p])
        rows = np.round(rng.dirichlet(np.ones(2), size=2), 4)  # [parent value][value]
        tables.append(rows.T.reshape(-1).tolist())
    with open(path, "w") as f:
        f.write('<?xml version="1.0" encoding="UTF-8"?>\n<BIF>\n<NETWORK>\n<NAME>tie</NAME>\n')
        for i in range(n):
            f.write("<VARIABLE>\n<NAME>X%d</NAME>\n<TYPE>discrete</TYPE>\n<VALUE>s0</VALUE>\n<VALUE>s1</VALUE>\n"
                    "</VARIABLE>\n" % i)
        for i in range(n):
            f.write("<PROBABILITY>\n<FOR>X%d</FOR>\n" % i)
            for q in parents[i]:
                f.write("<GIVEN>X%d</GIVEN>\n" % q)
            f.write("<TABLE>%s </TABLE>\n</PROBABILITY>\n" % " ".join("%.4f" % x for x in tables[i]))
        f.write("</NETWORK>\n</BIF>\n")
    return path


def synth_net_xml(name, path):
    from fastbn_amd import synth
    if name == "tie":
        return tie_network(path)
    synth.random_network(path=path, name=name, **SYNTH_NET_SPECS[name])
    return path


def synth_net_cases(name, xml):
    """The fixture's evidence cases (int8 [n][V]); tie: only X1..X8 observed (balanced counts tie)."""
    from fastbn_amd import synth
    net = synth.read_xmlbif(xml)
    if name == "tie":
        rng = np.random.Generator(np.random.PCG64(77))
        blocks = []
        for n, k, seed in SYNTH_NET_CASES[name]:
            ev = np.full((n, len(net[1])), -1, np.int8)
            for r in range(n):
                vs = rng.choice(np.arange(1, 9), size=min(k, 8) if r % 4 else r % 3 * 2, replace=False)
                ev[r, vs] = rng.integers(0, 2, size=vs.size)
            blocks.append(ev)
        return np.concatenate(blocks)
    return np.concatenate([synth.evidence_cases(net, n, k, seed=seed) for n, k, seed in SYNTH_NET_CASES[name]])


@pytest.fixture(scope="session")
def synth_nets(tmp_path_factory):
    """name -> {xml, ev, labels, marg} of the reference's own outputs (tests/golden/synth_nets)."""
    d = tmp_path_factory.mktemp("synth_nets")
    out = {}
    for name in ("bigdom", "wide", "tie"):
        xml = str(d / (name + ".xml"))
        with gzip.open(os.path.join(SYNTH_NETS, name + ".xml.gz"), "rb") as f, open(xml, "wb") as g:
            g.write(f.read())
        ev = np.load(os.path.join(SYNTH_NETS, name + ".ev.npy"))
        from fastbn_amd import synth
        dims = synth.read_xmlbif(xml)[1]
        lab, marg, _, _ = read_ref_marg(os.path.join(SYNTH_NETS, name + ".ref.marg.gz"), dims)
        out[name] = {"xml": xml, "ev": ev, "labels": lab, "marg": marg, "dims": dims}
    return out
