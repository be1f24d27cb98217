"""Config 5 (1000 variables x 100k samples) PC-stable through the C-ABI: median wall time per call
with level 0's Gram on the hand-written FP4 MFMA kernel (default), on the popcount kernel
(FBN_CI_GRAM_NO_MFMA) and on rocBLAS int8 (FBN_CI_GRAM_ROCBLAS, the previous round's path).  Each
variant runs in its own process; under rocprofv3 --kernel-trace --stats the per-kernel times of
all three land in one summary.  Usage: python tools/gram_timing.py [reps] [variant ...]"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

VARIANTS = {"mfma": {}, "popcount": {"FBN_CI_GRAM_NO_MFMA": "1"}, "rocblas": {"FBN_CI_GRAM_NO_MFMA": "1",
                                                                           "FBN_CI_GRAM_ROCBLAS": "1"}}


def run(reps, name):
    import fastbn_amd as F
    from fastbn_amd import synth
    cols, dims = synth.config5_dataset()
    ci = F.IndependenceTest(F.Dataset(columns=cols, dims=dims))
    pc = F.PCStable(0.05, 5)
    for _ in range(3):
        r = pc.StructLearnCompData(ci)
    ci.set_kernel_timing(False)
    h = ctypes.c_void_p()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        F.lib.fbn_pc_stable(ci._h, 0.05, 5, 1, ctypes.byref(h))
        t.append(time.perf_counter() - t0)
        F.lib.fbn_pc_result_destroy(h)
    print(f"{name}: median {1e3 * np.median(t):.3f} ms  min {1e3 * np.min(t):.3f} ms  "
          f"tests {r.tests_per_level.tolist()} edges {len(r.edges)}", flush=True)


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    names = sys.argv[2:] or list(VARIANTS)
    if os.environ.get("_GRAM_CHILD"):
        run(reps, names[0])
    else:
        for n in names:
            env = dict(os.environ, _GRAM_CHILD="1", **VARIANTS[n])
            subprocess.run([sys.executable, __file__, str(reps), n], check=True, env=env)
