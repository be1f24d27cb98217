"""Time the JT kernel for several persistent-wave settings in one process (interleaved rounds)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

xml = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
k = int(sys.argv[3]) if len(sys.argv) > 3 else 7
configs = [tuple(int(y) for y in x.split(":")) for x in
           (sys.argv[4] if len(sys.argv) > 4 else "0:1,0:2,0:3,0:4,0:6,0:8,2:2,1:8").split(",")]  # variant:waves
net = synth.read_xmlbif(xml)
ev = synth.evidence_cases(net, n, k, seed=1)
jt = F.JunctionTree(F.Network(xml), device=0)
print(jt.info, flush=True)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
res = {w: [] for w in configs}
for rnd in range(5):
    for w in configs:
        jt.set_variant(w[0])
        jt.set_waves_per_cu(w[1])
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), s)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), s)
        b.record()
        torch.cuda.synchronize()
        res[w].append(a.elapsed_time(b) / 3)
for w in configs:
    ms = float(np.median(res[w]))
    print(f"variant {w[0]} waves/CU {w[1]:3d}: {ms:8.3f} ms  {n / ms / 1e3:10.3f} Mcases/s  "
          f"{jt.info['algorithmic_bytes_per_case'] * n / ms / 1e6:8.1f} GB/s algorithmic", flush=True)
