"""Diagnostic: per-entry-pass cost of the streamed kernel (variant 4) on ALARM (constant data and
messages cache-resident) vs the Munin-like network.  virt_compare.py [cases]"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
nets = [("alarm", os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml"), 7)]
path = "/tmp/munin_like_cmp.xml"
synth.random_network(1041, seed=1041, window=12, path=path, name="munin_like")
nets.append(("munin_like", path, 208))
for name, xml, k in nets:
    net = synth.read_xmlbif(xml)
    ev = synth.evidence_cases(net, n, k, seed=1)
    jt = F.JunctionTree(F.Network(xml), device=0)
    d_ev = torch.from_numpy(ev).cuda()
    d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
    d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
    for v in (4, 1):
        jt.set_variant(v)
        ts = []
        for _ in range(4):
            jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
            ts.append(jt.last_kernel_ms())
        ms = float(np.median(ts[1:]))
        ent = jt.info["clique_entries"]
        print(f"{name} variant {v}: {ms:.2f} ms, {n / ms * 1e3:.0f} cases/s, "
              f"{ms * 1e6 / (n / 64) / ent:.3f} ns per wave-entry", flush=True)
