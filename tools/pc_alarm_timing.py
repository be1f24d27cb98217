"""Breakdown of one PC-stable run on alarm_s5000 (resident column store): wall / driver / kernels."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402

ds = F.Dataset(os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt"))
ci = F.IndependenceTest(ds)
pc = F.PCStable(0.05, 1000)
for _ in range(3):
    pc.StructLearnCompData(ci)
w, d, k = [], [], []
for _ in range(20):
    t0 = time.perf_counter()
    pc.StructLearnCompData(ci)
    w.append(time.perf_counter() - t0)
    d.append(pc.total_s)
    k.append(pc.kernel_s)
print(f"wall {1e3 * np.median(w):.3f} ms  driver {1e3 * np.median(d):.3f} ms  kernels {1e3 * np.median(k):.3f} ms  "
      f"launched {pc.launched_per_level.tolist()}")
