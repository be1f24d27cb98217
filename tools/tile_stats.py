"""Static statistics of the tiled JT program (variant 5) for a network: per-wave store size, wave
steps and factor loads by kind (LDS / wave store), and how often consecutive R steps of a pass read
the same factor row (the reuse a step-to-step select could exploit).  Host only:
tools/tile_stats.py [xml] (default: the seeded Munin-like network)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import fastbn_amd as F  # noqa: E402
import tile_emulator as TE  # noqa: E402
from fastbn_amd import synth  # noqa: E402

if len(sys.argv) > 1:
    xml = sys.argv[1]
else:
    xml = "/tmp/munin_like_once.xml"
    synth.random_network(1041, seed=1041, window=12, path=xml, name="munin_like")
jt = F.JunctionTree(F.Network(xml), device=-1)
passes, tab, iv, geo = jt.tile_program()
C = geo["cases_per_wave"]
print("store rows", geo["store_rows"], "-> per wave", geo["store_rows"] * C * 8 / 1e6, "MB; per case",
      geo["store_rows"] * 8 / 1e3, "kB; tab", len(tab) * 4 / 1e6, "MB")
steps = {"lds": 0, "glob": 0, "mixed": 0}
ld = {"lds": 0, "glob": 0, "glob_reuse": 0, "lds_reuse": 0}
kinds = {}
for prow in passes:
    P = dict(zip(TE.F, (int(x) for x in prow)))
    nf, nR = P["nf"], P["nRo"] * P["nRi"]
    ws = P["rounds"] * nR
    steps["lds" if P["nl"] == nf else "glob" if P["nl"] == 0 else "mixed"] += ws
    kinds[P["kind"]] = kinds.get(P["kind"], 0) + ws
    RS = nf + 2
    st = tab[P["st_off"]:P["st_off"] + nR * RS].reshape(nR, RS)
    for j in range(nf):
        lds = j < P["nl"]
        same = np.count_nonzero(st[:, j] & 1)
        key = "lds" if lds else "glob"
        ld[key] += ws
        ld[key + "_reuse"] += P["rounds"] * same
tot = sum(steps.values())
print("wave steps per 16 cases", tot, "by mode", steps, "by kind", kinds)
print("factor loads per 16 cases", ld, "glob reuse frac %.3f" % (ld["glob_reuse"] / max(1, ld["glob"])))
print("global factor loads per step %.2f, lds %.2f" % (ld["glob"] / tot, ld["lds"] / tot))

# factor spans (rows) of every pass, and the wave steps a per-factor LDS choice could cover
rowb = C * 8
spans = []
for prow in passes:
    P = dict(zip(TE.F, (int(x) for x in prow)))
    nf, nG, nRo, nRi = P["nf"], P["nG"], P["nRo"], P["nRi"]
    if nf == 0:
        continue
    g = tab[P["g_off"]:P["g_off"] + nG * (4 + nf)].reshape(nG, 4 + nf).astype(np.int64)
    nR = nRo * nRi
    st = tab[P["st_off"]:P["st_off"] + nR * (nf + 2)].reshape(nR, nf + 2).astype(np.int64)
    ws = P["rounds"] * nR
    rows = []
    for j in range(nf):
        off = (g[:, 4 + j][:, None] + (st[None, :, j] & ~1)).reshape(-1)
        rows.append(int((off.max() - off.min()) // rowb + 1))
    spans.append((ws, rows, P["nl"], P["kind"]))
for budget in (48, 64, 96, 128, 192, 256):
    cov = 0
    tot_f = 0
    for ws, rows, mode, kind in spans:
        left = budget
        for r in sorted(rows):
            tot_f += ws
            if r <= left:
                left -= r
                cov += ws
    print(f"budget {budget:4d} rows ({budget * rowb // 1024} KB): LDS share of factor loads {cov / tot_f:.3f}")
big = sorted(spans, key=lambda x: -x[0])[:15]
for ws, rows, mode, kind in big:
    print(ws, rows, mode, kind)
