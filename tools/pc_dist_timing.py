"""Diagnostic: config 5 through fbn_pc_stable vs the distributed session at world size 1."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fastbn_amd as F  # noqa: E402
from fastbn_amd import pc_dist, synth  # noqa: E402

cols, dims = synth.config5_dataset()
ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
F.PCStable(0.05, 6).StructLearnCompData(ci)
ci.set_kernel_timing(False)
h = ctypes.c_void_p()
for name, fn in (("fbn_pc_stable", lambda: F.lib.fbn_pc_stable(ci._h, 0.05, 6, 1, ctypes.byref(h))),
                 ("session w1", lambda: pc_dist.pc_stable_distributed(ci, 1000, 0.05, 6))):
    t = []
    for _ in range(7):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    print(f"{name}: median {1e3 * np.median(t):.2f} ms  min {1e3 * min(t):.2f} ms", flush=True)
os.environ["FBN_PC_TIMING"] = "1"
pc_dist.pc_stable_distributed(ci, 1000, 0.05, 6)
