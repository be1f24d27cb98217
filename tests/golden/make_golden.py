#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ from the *reference itself*.

TEST INFRASTRUCTURE -- runs only in the build container, where /root/reference exists.  It
  1. builds oracle/_ref/ref_dump (unmodified reference sources + our harness, oracle/Makefile),
  2. copies the reference's ALARM data files (public bnlearn benchmark data the reference ships
     under dataset/alarm/) into tests/golden/alarm/,
  3. writes a seeded synthetic evidence set (LIBSVM, same format as testing_alarm_1k_p20) and a
     seeded list of CI tests,
  4. runs the reference on them and stores its outputs as fixtures:
       alarm_1k.plan / .init      junction-tree plan + initial potentials (JunctionTree ctor)
       alarm_1k.marg.gz           per-case label + marginals for the 1000 shipped test cases
       alarm_rand.marg.gz         the same for the synthetic evidence set
       alarm_s5000.ci.gz          reference Counts2D/Counts3D tables for the CI test list
       alarm_shd.json             reference BNSLComparison::GetSHD for seeded learned graphs
                                  (perturbations of ALARM's DAG: undirected / reversed / dropped /
                                  added edges) against alarm.bif
No reference source text is copied; only data files and the reference's outputs.
"""
import gzip
import os
import random
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FBN_REFERENCE", "/root/reference")
DATA = os.path.join(REF, "dataset", "alarm")
OUT = os.path.join(HERE, "alarm")


def run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)


def gz(src, dst):
    with open(src, "rb") as f, gzip.GzipFile(dst, "wb", compresslevel=9, mtime=0) as g:
        shutil.copyfileobj(f, g)
    os.remove(src)


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present; fixtures are committed, nothing to do")
    run(["make", "-C", os.path.join(REPO, "oracle"), "ref"])
    ref_dump = os.path.join(REPO, "oracle", "_ref", "ref_dump")
    os.makedirs(OUT, exist_ok=True)
    for f in ["alarm.xml", "alarm.bif", "testing_alarm_1k_p20", "alarm_1k_pt", "alarm_s5000.txt"]:
        shutil.copyfile(os.path.join(DATA, f), os.path.join(OUT, f))

    # 1) shipped test cases
    pre = os.path.join(OUT, "alarm_1k")
    run([ref_dump, "jt", os.path.join(OUT, "alarm.xml"), os.path.join(OUT, "testing_alarm_1k_p20"),
         os.path.join(OUT, "alarm_1k_pt"), pre])
    gz(pre + ".marg", pre + ".marg.gz")

    # 2) synthetic evidence: 0..36 observed vars (var 0 is the query and never observed),
    #    including the empty and the all-observed patterns
    dims = [2, 3, 3, 2, 3, 2, 3, 2, 3, 3, 2, 3, 2, 2, 3, 4, 2, 4, 2, 3, 3, 3, 2, 2, 3, 4, 2, 3, 3, 4,
            4, 4, 3, 2, 3, 3, 3]
    rng = random.Random(20250131)
    lines = []
    for c in range(300):
        k = 0 if c == 0 else 36 if c == 1 else rng.randint(0, 36)
        vs = rng.sample(range(1, 37), k)
        feats = " ".join(f"{v}:{rng.randrange(dims[v])}" for v in vs)
        lines.append(f"{rng.randrange(2)} {feats}".rstrip() + " \n")
    rand_set = os.path.join(OUT, "rand_evidence.libsvm")
    with open(rand_set, "w") as f:
        f.writelines(lines)
    # the tree is built after loading testing_alarm_1k_p20 (same heap history as run 1, hence the
    # same pointer-ordered tree), then the synthetic cases are evaluated on it
    pre = os.path.join(HERE, "alarm_rand")
    run([ref_dump, "jt", os.path.join(OUT, "alarm.xml"), os.path.join(OUT, "testing_alarm_1k_p20"), "-", pre,
         "0", rand_set])
    gz(pre + ".marg", pre + ".marg.gz")
    for ext in (".plan", ".init"):
        same = open(pre + ext).read() == open(os.path.join(OUT, "alarm_1k" + ext)).read()
        assert same, "reference tree differs between runs (heap-address order)"
        os.remove(pre + ext)
    for ext in (".plan", ".init"):
        shutil.move(os.path.join(OUT, "alarm_1k" + ext), os.path.join(HERE, "alarm_1k" + ext))
    shutil.move(os.path.join(OUT, "alarm_1k.marg.gz"), os.path.join(HERE, "alarm_1k.marg.gz"))

    # 3) CI tests: every level-0 pair plus seeded conditional tests with |Z| = 1..4
    tests = [(x, y, []) for x in range(37) for y in range(x + 1, 37)]
    for _ in range(400):
        d = rng.randint(1, 4)
        xs = rng.sample(range(37), d + 2)
        x, y = sorted(xs[:2])
        tests.append((x, y, sorted(xs[2:])))
    tfile = os.path.join(HERE, "alarm_s5000.tests")
    with open(tfile, "w") as f:
        for x, y, z in tests:
            f.write(" ".join(map(str, [x, y] + z)) + "\n")
    ci = os.path.join(HERE, "alarm_s5000.ci")
    run([ref_dump, "ci", os.path.join(OUT, "alarm_s5000.txt"), tfile, ci])
    gz(ci, ci + ".gz")
    os.remove(tfile)

    # 4) SHD: seeded learned graphs scored by the reference's own GetSHD
    import json
    names, arcs = [], []
    for line in open(os.path.join(OUT, "alarm.bif")):
        t = line.strip()
        if t.startswith("variable "):
            names.append(t.split()[1])
        elif t.startswith("probability") and "|" in t:
            inner = t[t.index("(") + 1:t.index(")")]
            child, parents = inner.split("|")
            for p in parents.split(","):
                arcs.append((names.index(p.strip()), names.index(child.strip())))
    cases = []
    lfile = os.path.join(HERE, "learned.tmp")
    for k in range(40):
        g = {}
        for a, b in arcs:
            u = rng.random()
            if u < 0.1:
                continue  # dropped
            g[(min(a, b), max(a, b))] = (b, a, 1) if u < 0.25 else (min(a, b), max(a, b), 0) if u < 0.5 else (a, b, 1)
        for _ in range(rng.randint(0, 6)):  # spurious edges
            a, b = sorted(rng.sample(range(37), 2))
            if (a, b) not in g:
                g[(a, b)] = (a, b, 0) if rng.random() < 0.5 else ((a, b, 1) if rng.random() < 0.5 else (b, a, 1))
        edges = list(g.values())
        rng.shuffle(edges)
        with open(lfile, "w") as f:
            for e in edges:
                f.write("%d %d %d\n" % e)
        out = subprocess.run([ref_dump, "shd", os.path.join(OUT, "alarm.bif"), lfile], check=True,
                             capture_output=True, text=True).stdout
        cases.append({"edges": edges, "shd": int(out.split()[1])})
    os.remove(lfile)
    with open(os.path.join(HERE, "alarm_shd.json"), "w") as f:
        json.dump(cases, f, separators=(",", ":"))
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
