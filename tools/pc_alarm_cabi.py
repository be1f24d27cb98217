"""PC-stable on alarm_s5000 through the C-ABI call (as bench.py times it): median wall of
fbn_pc_stable (skeleton + orientation), the driver's skeleton time and the kernel time.
pc_alarm_cabi.py [runs] [label]"""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 50
label = sys.argv[2] if len(sys.argv) > 2 else ""
ds = F.Dataset(os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt"))
ci = F.IndependenceTest(ds)
pc = F.PCStable(0.05, 1000)
for _ in range(3):
    pc.StructLearnCompData(ci)
kern = pc.kernel_s
ci.set_kernel_timing(False)
h = ctypes.c_void_p()
w, drv = [], []
for _ in range(runs):
    t0 = time.perf_counter()
    F.lib.fbn_pc_stable(ci._h, 0.05, 1000, 1, ctypes.byref(h))
    w.append(time.perf_counter() - t0)
    r = F.PCResult(h)  # destroys the handle when dropped
    drv.append(r.total_s)
    del r
ci.set_kernel_timing(True)
print(f"{label}: C-ABI call {1e3 * np.median(w):.3f} ms (min {1e3 * np.min(w):.3f}), skeleton driver "
      f"{1e3 * np.median(drv):.3f} ms, kernels {1e3 * kern:.3f} ms, tests {pc.num_ci_test}, edges {len(pc.edges)}",
      flush=True)
