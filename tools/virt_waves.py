"""Diagnostic: streamed JT kernel (variant 4) time on the Munin-like network vs resident waves per CU."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
waves = [int(w) for w in (sys.argv[2] if len(sys.argv) > 2 else "4,8,12,16").split(",")]
path = "/tmp/munin_like_w.xml"
synth.random_network(1041, seed=1041, window=12, path=path, name="munin_like")
ev = synth.evidence_cases(synth.read_xmlbif(path), n, 208, seed=20250131)
jt = F.JunctionTree(F.Network(path), device=0)
jt.set_variant(4)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
for w in waves:
    jt.set_waves_per_cu(w)
    ts = []
    for _ in range(3):
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
        ts.append(jt.last_kernel_ms())
    ms = float(np.median(ts))
    print(f"waves/CU {w}: {ms:.1f} ms, {n / ms * 1e3:.0f} cases/s", flush=True)
