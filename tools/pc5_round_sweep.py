"""Config 5 level-1 round schedule sweep with the information screen on: FBN_PC_ROUND0 (first chunk =
ROUND0 / E candidate sets per edge, <= 32) x FBN_PC_GROWTH; median ms per C-ABI call, launched tests,
fixture check.  usage: pc5_round_sweep.py [reps]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import fastbn_amd as F  # noqa: E402
from conftest import pc_digest  # noqa: E402
from fastbn_amd import synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 15
cols, dims = synth.config5_dataset(1000, 100000)
ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
ref = json.load(open(os.path.join(REPO, "tests", "golden", "pc_c5.json")))
for r0, gr in [(8192, 2), (60000, 2), (120000, 2), (240000, 2), (120000, 4), (240000, 4), (1000000, 2), (8192, 2)]:
    os.environ["FBN_PC_ROUND0"], os.environ["FBN_PC_GROWTH"] = str(r0), str(gr)
    r = F.PCStable(0.05, 6).StructLearnCompData(ci)
    ok = (r.tests_per_level.tolist() == ref["tests_per_level"] and
          pc_digest(r.edges, r.sepset) == {k: ref[k] for k in ("edges_sha256", "sepsets_sha256")})
    ci.set_kernel_timing(False)
    h = ctypes.c_void_p()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        F.lib.fbn_pc_stable(ci._h, 0.05, 6, 1, ctypes.byref(h))
        t.append(time.perf_counter() - t0)
        F.lib.fbn_pc_result_destroy(h)
    ci.set_kernel_timing(True)
    print(f"round0 {r0} growth {gr}: {1e3 * np.median(t):.3f} ms, launched {r.launched_per_level.tolist()[1]}, fixture {ok}",
          flush=True)
