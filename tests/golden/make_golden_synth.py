#!/usr/bin/env python3
"""Fixtures that pin BASELINE configs 4 and 5 at their real network / dataset sizes.

TEST INFRASTRUCTURE -- runs in the build container.

  munin_like/   config 4: the seeded Munin-like network (1041 variables) as
                XMLBIF, 32 seeded evidence cases (208 observed variables each, LIBSVM), and the
                *reference's own* outputs on them (oracle/_ref/ref_dump jt: the unmodified
                reference JunctionTree compiled in place): per-case label + 17-digit marginals
                (ref.marg.gz) and the reference's junction-tree plan (ref.plan.gz).
  pc_c5.ci.gz   config 5: the reference's own Counts2D / Counts3D tables (pc_c5_ci below)
  synth_nets/   networks beyond ALARM / Munin-like (tests/conftest.py SYNTH_NET_SPECS, tie_network):
                state counts up to 21, a 12-variable clique, symmetric CPTs whose query marginals
                tie; seeded evidence cases (.ev.npy) and the reference's own labels + marginals
  pc_c5.json    config 5: PC-stable (depth 6, alpha 0.05) on the seeded 1000-variable x 100k-sample
                dataset, run by the CPU restatement (oracle/pc_oracle.cpp; the reference's
                PCStable/IndependenceTest cannot be compiled here: stats/gcem absent): tests per
                level, edge count and digests of the edge list and of the sepsets, plus the digest
                of the column store so the GPU test knows it regenerated the same data.

No reference source text is copied; only its outputs on our generated inputs.
"""
import gzip
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))

MUNIN_CASES = 32


def gz_write(path, data):
    with gzip.GzipFile(path, "wb", compresslevel=9, mtime=0) as g:
        g.write(data if isinstance(data, bytes) else data.encode())


def munin_like():
    from fastbn_amd import synth
    out = os.path.join(HERE, "munin_like")
    os.makedirs(out, exist_ok=True)
    ref_dump = os.path.join(REPO, "oracle", "_ref", "ref_dump")
    if not os.path.exists(ref_dump):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    with tempfile.TemporaryDirectory() as td:
        xml = os.path.join(td, "munin_like.xml")
        synth.random_network(1041, seed=1041, window=12, path=xml, name="munin_like")
        net = synth.read_xmlbif(xml)
        ev = synth.evidence_cases(net, MUNIN_CASES, 208, seed=20250131)
        lib = os.path.join(td, "ev.libsvm")
        with open(lib, "w") as f:
            for r in ev:
                f.write("0 " + " ".join(f"{v}:{r[v]}" for v in range(r.size) if r[v] >= 0) + " \n")
        pre = os.path.join(td, "ref")
        subprocess.run([ref_dump, "jt", xml, lib, "-", pre, str(MUNIN_CASES)], check=True,
                       stdout=subprocess.DEVNULL)
        gz_write(os.path.join(out, "munin_like.xml.gz"), open(xml, "rb").read())
        gz_write(os.path.join(out, "ev.libsvm.gz"), open(lib, "rb").read())
        gz_write(os.path.join(out, "ref.marg.gz"), open(pre + ".marg", "rb").read())
        gz_write(os.path.join(out, "ref.plan.gz"), open(pre + ".plan", "rb").read())


MUNIN_EXTRA = (16, 0), (16, 52), (16, 208), (16, 520)  # (cases, observed variables): 64 cases


def munin_like_extra():
    """munin_like/extra_*: 64 more cases of the same network at 0 / 52 / 208 / 520 observed variables
    (seed 7), with the reference's labels and 17-digit marginals -- the fast-order tiled kernel (the
    Munin-class default) against the reference beyond the 32 base cases."""
    import numpy as np
    from fastbn_amd import synth
    out = os.path.join(HERE, "munin_like")
    ref_dump = os.path.join(REPO, "oracle", "_ref", "ref_dump")
    if not os.path.exists(ref_dump):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    with tempfile.TemporaryDirectory() as td:
        xml = os.path.join(td, "munin_like.xml")
        synth.random_network(1041, seed=1041, window=12, path=xml, name="munin_like")
        net = synth.read_xmlbif(xml)
        ev = np.concatenate([synth.evidence_cases(net, n, k, seed=7 + k) for n, k in MUNIN_EXTRA])
        n = ev.shape[0]
        lib = os.path.join(td, "ev.libsvm")
        with open(lib, "w") as f:
            for r in ev:
                f.write("0 " + " ".join(f"{v}:{r[v]}" for v in range(r.size) if r[v] >= 0) + " \n")
        pre = os.path.join(td, "ref")
        subprocess.run([ref_dump, "jt", xml, lib, "-", pre, str(n)], check=True, stdout=subprocess.DEVNULL)
        gz_write(os.path.join(out, "extra_ev.libsvm.gz"), open(lib, "rb").read())
        gz_write(os.path.join(out, "extra_ref.marg.gz"), open(pre + ".marg", "rb").read())


def pc_c5():
    import numpy as np
    import oracle as O
    from conftest import pc_digest
    from fastbn_amd import synth
    cols, dims = synth.config5_dataset()
    t0 = time.time()
    r = O.OracleDataset(columns=cols, dims=dims).pc_stable(0.05, 6, 1)
    secs = time.time() - t0
    import hashlib
    rec = {"nvars": int(cols.shape[0]), "nsamples": int(cols.shape[1]), "depth": 6, "alpha": 0.05,
           "columns_sha256": hashlib.sha256(np.ascontiguousarray(cols).tobytes()).hexdigest(),
           "dims": dims.tolist(),
           "tests_per_level": r["tests_per_level"], "num_ci_test": r["num_ci_test"],
           "num_edges": len(r["edges"]), "num_sepsets": len(r["sepset"]),
           **pc_digest(r["edges"], r["sepset"]),
           "oracle_seconds": round(secs, 1)}
    with open(os.path.join(HERE, "pc_c5.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print("pc_c5:", {k: v for k, v in rec.items() if k != "dims"})


# per level of the config-5 run: how many of the tests the reference's sequential search runs are
# pinned (seeded sample of the restatement's log; deep levels have few tests and large tables)
C5CI_PER_LEVEL = {0: 256, 1: 256, 2: 192, 3: 128, 4: 96, 5: 30}


def pc_c5_ci():
    """pc_c5.ci.gz: the UNMODIFIED reference's Counts2D / Counts3D::FillTable (src/CellTable.cpp,
    compiled in place into oracle/_ref/ref_dump) on a seeded sample of the CI tests a config-5 run
    performs at every level 0-5 -- the tests come from the restatement's log of the full run
    (oracle/pc_oracle.cpp, the order the reference's sequential search would run them), the counts
    and the per-column FNV-1a hashes from the reference's own code reading the same column store."""
    import random

    import numpy as np
    import oracle as O
    from fastbn_amd import synth
    ref_dump = os.path.join(REPO, "oracle", "_ref", "ref_dump")
    if not os.path.exists(ref_dump):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    cols, dims = synth.config5_dataset()
    t0 = time.time()
    r = O.OracleDataset(columns=cols, dims=dims).pc_stable(0.05, 6, 1, keep_log=True)
    print("restatement run: %.1f s, %d logged tests" % (time.time() - t0, len(r["log"])))
    by_level = {}
    for t in r["log"]:
        by_level.setdefault(t[0], []).append(t)
    rng = random.Random(20251017)
    sample = []
    for d in sorted(by_level):
        tests = by_level[d]
        k = min(C5CI_PER_LEVEL.get(d, 32), len(tests))
        sample += [tests[i] for i in sorted(rng.sample(range(len(tests)), k))]
    with tempfile.TemporaryDirectory() as td:
        cpath = os.path.join(td, "c5.cols")
        with open(cpath, "wb") as f:
            import struct
            f.write(struct.pack("<iq", cols.shape[0], cols.shape[1]))
            f.write(np.asarray(dims, np.int32).tobytes())
            f.write(np.ascontiguousarray(cols, np.uint8).tobytes())
        tfile = os.path.join(td, "tests")
        with open(tfile, "w") as f:
            for t in sample:
                f.write(" ".join(map(str, [t[1], t[2]] + list(t[3]))) + "\n")
        out = os.path.join(td, "c5.ci")
        subprocess.run([ref_dump, "ci", "cols:" + cpath, tfile, out], check=True, stdout=subprocess.DEVNULL)
        gz_write(os.path.join(HERE, "pc_c5.ci.gz"), open(out, "rb").read())
    print("pc_c5.ci.gz: %d tests, per level %s" % (len(sample), {d: min(C5CI_PER_LEVEL.get(d, 32), len(v))
                                                             for d, v in sorted(by_level.items())}))


GRAM_PAIRS = 320  # per shape: a seeded sample of the test's pairs plus the tile-edge pairs


def gram_ragged():
    """gram_ragged.ci.gz: the UNMODIFIED reference's Counts2D::FillTable (src/CellTable.cpp:430-455,
    oracle/_ref/ref_dump ci) on the ragged-shape datasets of test_gpu_gram_mfma.py (conftest
    gram_dataset: leading-row counts not multiples of the 256-row Gram tile, sample counts not
    multiples of the 128-sample stage), one block per shape: `shape nvars N seed` then the ci dump."""
    import random
    import struct

    import numpy as np
    from conftest import GRAM_SHAPES, gram_dataset
    ref_dump = os.path.join(REPO, "oracle", "_ref", "ref_dump")
    if not os.path.exists(ref_dump):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    blocks = []
    for nvars, N, seed in GRAM_SHAPES:
        cols, dims, pairs = gram_dataset(nvars, N, seed)
        rng = random.Random(seed)
        idx = sorted(set(rng.sample(range(len(pairs) - 3), GRAM_PAIRS - 3)) | {len(pairs) - 3, len(pairs) - 2,
                                                                              len(pairs) - 1})
        with tempfile.TemporaryDirectory() as td:
            cpath = os.path.join(td, "g.cols")
            with open(cpath, "wb") as f:
                f.write(struct.pack("<iq", nvars, N))
                f.write(np.asarray(dims, np.int32).tobytes())
                f.write(np.ascontiguousarray(cols, np.uint8).tobytes())
            tfile = os.path.join(td, "tests")
            with open(tfile, "w") as f:
                for i in idx:
                    f.write("%d %d\n" % (pairs[i, 0], pairs[i, 1]))
            out = os.path.join(td, "g.ci")
            subprocess.run([ref_dump, "ci", "cols:" + cpath, tfile, out], check=True, stdout=subprocess.DEVNULL)
            blocks.append("shape %d %d %d\n" % (nvars, N, seed) + open(out).read())
    gz_write(os.path.join(HERE, "gram_ragged.ci.gz"), "".join(blocks))
    print("gram_ragged.ci.gz: %d shapes x %d pairs" % (len(GRAM_SHAPES), GRAM_PAIRS))


def synth_nets():
    """synth_nets/<name>.{xml.gz, ev.npy, ref.marg.gz} for name in bigdom / wide / tie: the XMLBIF,
    the evidence cases (conftest.synth_net_cases) and the UNMODIFIED reference's labels and 17-digit
    marginals on them (oracle/_ref/ref_dump jt)."""
    import numpy as np
    from conftest import SYNTH_NETS, synth_net_cases, synth_net_xml
    ref_dump = os.path.join(REPO, "oracle", "_ref", "ref_dump")
    if not os.path.exists(ref_dump):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    os.makedirs(SYNTH_NETS, exist_ok=True)
    for name in ("bigdom", "wide", "tie"):
        with tempfile.TemporaryDirectory() as td:
            xml = synth_net_xml(name, os.path.join(td, name + ".xml"))
            ev = synth_net_cases(name, xml)
            lib = os.path.join(td, "ev.libsvm")
            with open(lib, "w") as f:
                for r in ev:
                    f.write("0 " + " ".join(f"{v}:{r[v]}" for v in range(r.size) if r[v] >= 0) + " \n")
            pre = os.path.join(td, "ref")
            t0 = time.time()
            subprocess.run([ref_dump, "jt", xml, lib, "-", pre, str(len(ev))], check=True, stdout=subprocess.DEVNULL)
            gz_write(os.path.join(SYNTH_NETS, name + ".xml.gz"), open(xml, "rb").read())
            np.save(os.path.join(SYNTH_NETS, name + ".ev.npy"), ev)
            gz_write(os.path.join(SYNTH_NETS, name + ".ref.marg.gz"), open(pre + ".marg", "rb").read())
            print("synth_nets/%s: %d cases, reference %.1f s" % (name, len(ev), time.time() - t0))


if __name__ == "__main__":
    which = sys.argv[1:] or ["munin", "munin_extra", "c5", "c5ci", "gram", "synth_nets"]
    if "munin" in which:
        munin_like()
    if "munin_extra" in which:
        munin_like_extra()
    if "c5" in which:
        pc_c5()
    if "c5ci" in which:
        pc_c5_ci()
    if "gram" in which:
        gram_ragged()
    if "synth_nets" in which:
        synth_nets()
