"""Diagnostic: does the plan-specialized JT kernel gain from more waves per SIMD?  On a network
small enough that the kernel needs few registers, time variant 3 at 4 / 8 / 16 / 32 waves per CU
(1 / 2 / 4 / 8 per SIMD) for the same cases: tools/jt_occupancy.py [nvars] [ncases]."""
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

nv = int(sys.argv[1]) if len(sys.argv) > 1 else 37
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
path = os.path.join(tempfile.mkdtemp(), "small.xml")
synth.random_network(nv, seed=3, window=3, parent_probs=(0.7, 0.3), dom=(2, 3), path=path)
net = F.Network(path)
ev = net.evidence_cases(n, max(1, nv // 5), 1)
jt = F.JunctionTree(net, device=0)
print({k: jt.info[k] for k in ("num_cliques", "clique_entries", "specialized_eligible")}, flush=True)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
jt.set_evidence_check(False)
jt.set_variant(3)
res = {}
for rnd in range(4):
    for w in (4, 8, 16, 32):
        jt.set_waves_per_cu(w)
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
        b.record()
        torch.cuda.synchronize()
        res.setdefault(w, []).append(a.elapsed_time(b) / 3)
for w, v in res.items():
    print(f"waves/CU {w:3d}: {np.median(v):.3f} ms  {n / np.median(v) / 1e3:.2f} Mcases/s", flush=True)
