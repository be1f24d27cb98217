"""TEST INFRASTRUCTURE: executes the tiled kernel's program (variant 5, fastbn_amd/csrc/jt_tile.hip,
tables from jt_tile_plan.cpp via fbn_jt_tile_program) on the host with numpy, one case at a time,
so that the plan compiler's G / R records, factor offsets, LDS staging records, output bins and
marginal sources are checked against the oracle without a GPU (tests/test_host.py).  Same algebra
as the kernel (entry = G-part + R-part; w = init * prod factors, 0 against the evidence; output
bins U times sigma = 1 / prod of the factors' scales -> un-normalized messages with a scale row,
marginals from old * U), different summation order (numpy), so results agree with the oracle to
~1e-14, not bit for bit.  Never used by the product path."""
import numpy as np

# JtTPass field order (jt_program.h)
F = ["kind", "clique", "nf", "nl", "nG", "rounds", "nRo", "nRi", "g_off", "o_off", "i_off", "nE", "nbins",
     "dest_row", "col_row", "bdig_off", "nmv", "mv_off", "iv_off", "nv", "vars_off", "gfields", "ofields", "first",
     "nstage", "stage_off", "et_off", "st_off", "fsc_off", "dest_sc", "col_sc", "split", "chunk"]
COL, DIS, MARG = 0, 1, 2


def run_case(prog, ev_row, sum_dom, lds_bytes=1 << 20):
    """One evidence case (int8 [V], -1 unobserved) -> (label, marginals [sum_dom])."""
    passes, tab, iv, geo = prog
    C = geo["cases_per_wave"]
    row_b = C * 8  # bytes per message row (the kernel's [entry][C cases] layout; this case is case 0)
    store = np.zeros(geo["store_rows"])
    lds = np.zeros(lds_bytes // 8)
    out = np.zeros(sum_dom)
    label = None
    M = W = 0
    for prow in passes:
        P = dict(zip(F, (int(x) for x in prow)))
        P["gfields"] &= 0xFFFFFFFF
        P["ofields"] &= 0xFFFFFFFF
        nf = P["nf"]
        if P["first"]:
            M = W = 0
            for j in range(P["nv"]):
                var, sh, fm = tab[P["vars_off"] + 3 * j:P["vars_off"] + 3 * j + 3]
                x = int(ev_row[var])
                if x >= 0:
                    M |= int(fm) << int(sh)
                    W |= x << int(sh)
            for k in range(P["nstage"]):
                src, rows, dst = (int(v) for v in tab[P["stage_off"] + 3 * k:P["stage_off"] + 3 * k + 3])
                lds[dst // 8:dst // 8 + rows * C:C] = store[src:src + rows]
        mv = [tuple(int(v) for v in tab[P["mv_off"] + 5 * m:P["mv_off"] + 5 * m + 5]) for m in range(P["nmv"])]
        sig = 1.0 / np.prod([store[int(r)] for r in tab[P["fsc_off"]:P["fsc_off"] + nf]])
        if P["kind"] == MARG and all(int(ev_row[v]) >= 0 for v, *_ in mv):
            for var, off, dim, _, _ in mv:
                out[off:off + dim] = 0.0
            continue
        nG, nRo, nRi = P["nG"], P["nRo"], P["nRi"]
        g = tab[P["g_off"]:P["g_off"] + nG * (4 + nf)].reshape(nG, 4 + nf).astype(np.int64)
        ro = tab[P["o_off"]:P["o_off"] + nRo * (4 + nf)].reshape(nRo, 4 + nf).astype(np.int64)
        ri = tab[P["i_off"]:P["i_off"] + nRi * (2 + nf)].reshape(nRi, 2 + nf).astype(np.int64)
        # R record (o, i) = outer part + inner part (inner entry offsets are in bytes)
        r = np.zeros((nRo * nRi, 2 + nf), np.int64)
        r[:, 0] = (ro[:, 0:1] + ri[None, :, 0] // 8).reshape(-1)
        r[:, 1] = ((ro[:, 1:2] & 0xFFFFFFFF) | (ri[None, :, 1] & 0xFFFFFFFF)).reshape(-1)
        for j in range(nf):
            r[:, 2 + j] = (ro[:, 4 + j:5 + j] + ri[None, :, 2 + j]).reshape(-1)
        otab = ro[:, 2]
        e = g[:, 0:1] + r[None, :, 0]
        dw = (g[:, 1:2] & 0xFFFFFFFF) | (r[None, :, 1] & 0xFFFFFFFF)
        ok = ((dw ^ W) & M) == 0
        x = iv[P["iv_off"] + e].copy()
        for j in range(nf):
            off = g[:, 4 + j:5 + j] + r[None, :, 2 + j]
            in_lds = j < P["nl"]
            x *= lds[off // 8] if in_lds else store[off // row_b]
        x[~ok] = 0.0
        acc = x.reshape(nG, nRo, nRi).sum(axis=2)
        xidx = g[:, 2:3] + otab[None, :]
        nb, nE = P["nbins"], P["nE"]
        part = np.zeros(nb * nE)
        part[xidx.reshape(-1)] = acc.reshape(-1)
        v = part.reshape(nb, nE).sum(axis=1) * sig
        if P["kind"] != MARG:  # un-normalized message U, scale sum U
            store[P["dest_row"]:P["dest_row"] + nb] = v
            store[P["dest_sc"]] = v.sum()
        if P["kind"] == DIS:
            # the child's own Collect message `old` (not a factor of the pass) cancels in the
            # reference's (U / S') / old; the marginal bins are old * U
            v = store[P["col_row"]:P["col_row"] + nb] * v
        bd = tab[P["bdig_off"]:P["bdig_off"] + nb].astype(np.int64) & 0xFFFFFFFF
        for var, off, dim, sh, fm in mv:
            if int(ev_row[var]) >= 0:
                out[off:off + dim] = 0.0
                continue
            dg = (bd >> sh) & fm
            a = np.array([v[dg == d].sum() for d in range(dim)])
            out[off:off + dim] = a / a.sum()
            if var == 0:
                label = int(np.argmax(out[off:off + dim]))
    return label, out


def run(prog, ev, sum_dom):
    labs, margs = [], []
    for row in ev:
        lab, m = run_case(prog, row, sum_dom)
        labs.append(-1 if lab is None else lab)
        margs.append(m)
    return np.array(labs, np.int32), np.stack(margs)
