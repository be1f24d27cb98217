"""Config 5 (1000 x 100k, levels 0-5) through the C-ABI call with and without the level-1
information screen (FBN_PC_NO_MISCREEN): per-call ms (median), counted / launched tests per level,
and the skeleton digest against tests/golden/pc_c5.json.  usage: pc5_screen_probe.py [reps]"""
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

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cols, dims = synth.config5_dataset(1000, 100000)
ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
ref = json.load(open(os.path.join(REPO, "tests", "golden", "pc_c5.json")))
for mode in ("screen", "noscreen", "screen"):
    if mode == "noscreen":
        os.environ["FBN_PC_NO_MISCREEN"] = "1"
    else:
        os.environ.pop("FBN_PC_NO_MISCREEN", None)
    pc = F.PCStable(0.05, 6)
    r = pc.StructLearnCompData(ci)
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
    print(f"{mode}: {1e3 * np.median(t):.3f} ms (min {1e3 * min(t):.3f}), kernel {1e3 * r.kernel_s:.3f} ms, "
          f"tests {r.tests_per_level.tolist()}, launched {r.launched_per_level.tolist()}, fixture {ok}, path {r.path}",
          flush=True)
