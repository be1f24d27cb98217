"""Per-op-type cycle breakdown of the LDS JT kernel (diagnostic s_memtime build)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
n = 100000
ev = synth.evidence_cases(synth.read_xmlbif(xml), n, 7, seed=1)
jt = F.JunctionTree(F.Network(xml), device=0)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
for w in (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,4").split(",")):
    jt.set_waves_per_cu(w)
    jt.op_cycles(True, read=False)
    jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
    torch.cuda.synchronize()
    ms = jt.last_kernel_ms()
    c = jt.op_cycles(False)
    tot = sum(c.values())
    print(f"waves/CU {w}: kernel {ms:.3f} ms (profiled)  total op cycles {tot:.3e}")
    for k, v in c.items():
        if v:
            print(f"   {k:7s} {v:14.3e}  {100 * v / tot:5.1f}%")
