"""ALARM-5000 (BASELINE config 3) through the C-ABI call (the device-resident search) with and
without the level-1 information screen (FBN_PC_NO_MISCREEN): median ms per call over `reps`, the
kernel time, counted / launched tests per level, edges.  usage: pc_alarm_screen_probe.py [reps]"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ci = F.IndependenceTest(F.Dataset(os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt")))
for mode in ("screen", "noscreen", "screen"):
    if mode == "noscreen":
        os.environ["FBN_PC_NO_MISCREEN"] = "1"
    else:
        os.environ.pop("FBN_PC_NO_MISCREEN", None)
    pc = F.PCStable(0.05, 1000)
    for _ in range(3):
        r = pc.StructLearnCompData(ci)
    ci.set_kernel_timing(False)
    h = ctypes.c_void_p()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        F.lib.fbn_pc_stable(ci._h, 0.05, 1000, 1, ctypes.byref(h))
        t.append(time.perf_counter() - t0)
        F.lib.fbn_pc_result_destroy(h)
    ci.set_kernel_timing(True)
    print(f"{mode}: {1e3 * np.median(t):.4f} ms (min {1e3 * min(t):.4f}), kernel {1e3 * r.kernel_s:.4f} ms, "
          f"tests {r.tests_per_level.tolist()}, launched {r.launched_per_level.tolist()}, edges {len(r.edges)}, "
          f"path {r.path}", flush=True)
