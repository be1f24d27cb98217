"""Munin-like JT: seeded 1041-node network, 20 % evidence; parity on a few
cases vs the oracle and timing of the interpreter variants.  munin_probe.py [ncases] [variants]"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
variants = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1").split(",")]
path = "/tmp/munin_like.xml"
t0 = time.time()
synth.random_network(1041, seed=1041, window=12, path=path, name="munin_like")
net = synth.read_xmlbif(path)
ev = synth.evidence_cases(net, n, 208, seed=20250131)
print(f"network + {n} cases generated in {time.time() - t0:.1f} s", flush=True)
t0 = time.time()
jt = F.JunctionTree(F.Network(path), device=0)
print(f"plan {time.time() - t0:.2f} s", jt.info, flush=True)
import oracle as O  # noqa: E402
k = min(n, 64)
t0 = time.time()
olab, omarg = O.OracleJT(path).infer(ev[:k])
print(f"oracle {k} cases {time.time() - t0:.2f} s", flush=True)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
for v in variants:
    jt.set_variant(v)
    jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
    torch.cuda.synchronize()
    ok = (d_lab[:k].cpu().numpy() == olab).all() and (d_marg[:k].cpu().numpy() == omarg).all()
    ts = []
    for _ in range(3):
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
        ts.append(jt.last_kernel_ms())
    ms = float(np.median(ts))
    print(f"variant {v}: bit-exact on {k} cases: {ok}; {ms:.2f} ms for {n} cases = {n / ms * 1e3:.0f} cases/s; "
          f"algorithmic {jt.info['algorithmic_bytes_per_case'] * n / ms / 1e6:.0f} GB/s", flush=True)
