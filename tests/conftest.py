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
