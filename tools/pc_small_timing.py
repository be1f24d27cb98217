"""ALARM-5000 PC-stable through the C-ABI (fbn_pc_stable): median wall time per call for the
device-resident search (pc_small.hip) and the host-driven level loop (FBN_PC_NO_SMALL), plus the
kernel time of one timed call.  Usage: python tools/pc_small_timing.py [reps]"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run(reps):
    import fastbn_amd as F
    ds = F.Dataset(os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt"))
    ci = F.IndependenceTest(ds)
    pc = F.PCStable(0.05, 1000)
    for _ in range(5):
        pc.StructLearnCompData(ci)
    kernel_ms = 1e3 * pc.kernel_s
    ci.set_kernel_timing(False)
    h = ctypes.c_void_p()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        F.lib.fbn_pc_stable(ci._h, 0.05, 1000, 1, ctypes.byref(h))
        t.append(time.perf_counter() - t0)
        F.lib.fbn_pc_result_destroy(h)
    mode = ("host-driven" if os.environ.get("FBN_PC_NO_SMALL") else
            "device-resident (cooperative)" if os.environ.get("FBN_PC_SMALL_COOP") else "device-resident (plain launch)")
    print(f"{mode}: "
          f"median {1e3 * np.median(t):.4f} ms  min {1e3 * np.min(t):.4f} ms  kernel {kernel_ms:.4f} ms  "
          f"tests {pc.tests_per_level.tolist()} launched {pc.launched_per_level.tolist()} edges {len(pc.edges)}",
          flush=True)


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    if os.environ.get("_PCST_CHILD"):
        run(reps)
    else:
        for extra in ({}, {"FBN_PC_SMALL_COOP": "1"}, {}, {"FBN_PC_SMALL_COOP": "1"}, {"FBN_PC_NO_SMALL": "1"}):
            env = dict(os.environ, _PCST_CHILD="1", **extra)
            subprocess.run([sys.executable, __file__, str(reps)], check=True, env=env)
        env = dict(os.environ, _PCST_CHILD="1", FBN_PC_TIMING="1")
        subprocess.run([sys.executable, __file__, "3"], check=True, env=env)
