"""Diagnostic: the multi-GPU PC session (fastbn_amd.pc_dist) at world size 1 on the config-5 dataset
(1000 vars x 100k samples, levels 0-5), per level: fbn_pc_dist_level / _run / _apply wall times,
then fbn_pc_dist_result; the single-GPU call beside it.  Last, medians of the raw C-ABI call
fbn_pc_stable against pc_stable_distributed (bench.py's `session_world1`).  FBN_PC_TIMING=1 adds the
driver's per-level host phase prints."""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import pc_dist, synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cols, dims = synth.config5_dataset(1000, 100_000)
ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
ci.set_kernel_timing(False)
for r in range(runs):
    pc = F.PCStable(0.05, 6)
    t0 = time.perf_counter()
    pc.StructLearnCompData(ci)
    single = time.perf_counter() - t0
    T = []
    t0 = time.perf_counter()
    sess = pc_dist.PCDistSession(1000, 0.05, 6, 1)
    while True:
        a = time.perf_counter()
        lv = sess.level(1, 0)
        if lv is None:
            break
        d, b, e, L = lv
        bb = time.perf_counter()
        rec = sess.run(ci, L)
        c = time.perf_counter()
        more = sess.apply(pc_dist._all_gather_fixed(rec, None))
        dd = time.perf_counter()
        T.append((d, e - b, L, bb - a, c - bb, dd - c))
        if not more:
            break
    a = time.perf_counter()
    res = sess.result()
    rs = time.perf_counter() - a
    tot = time.perf_counter() - t0
    same = res.edges == pc.edges and res.sepset == pc.sepset
    print(f"run {r}: single {single * 1e3:.3f} ms, session {tot * 1e3:.3f} ms (result {rs * 1e3:.3f} ms), same {same}",
          flush=True)
    for d, n, L, tl, tr, ta in T:
        print(f"   d={d} edges {n} rec {L}: level {tl * 1e3:.3f} run {tr * 1e3:.3f} apply {ta * 1e3:.3f} ms", flush=True)
    del res, sess, pc  # (the sepset dicts `same` built take ~10 ms to free: outside the timed windows)

h = ctypes.c_void_p()


def single_call():
    F.lib.fbn_pc_stable(ci._h, 0.05, 6, 1, ctypes.byref(h))
    return h


for name, fn, done in (("fbn_pc_stable", single_call, lambda r: F.lib.fbn_pc_result_destroy(r)),
                       ("session w1", lambda: pc_dist.pc_stable_distributed(ci, 1000, 0.05, 6), lambda r: None)):
    t = []
    for _ in range(9):
        t0 = time.perf_counter()
        out = fn()
        t.append(time.perf_counter() - t0)
        done(out)
        del out
    print(f"{name}: median {1e3 * np.median(t):.3f} ms  min {1e3 * min(t):.3f} ms", flush=True)
