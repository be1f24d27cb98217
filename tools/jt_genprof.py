"""Per-category cycle breakdown of the specialized JT kernel (run with FBN_JT_PROFILE=1)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
ev = synth.evidence_cases(synth.read_xmlbif(xml), n, 7, seed=1)
jt = F.JunctionTree(F.Network(xml), device=0)
jt.set_variant(3)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
jt.op_cycles(True, read=False)
jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
torch.cuda.synchronize()
c = jt.op_cycles(False)
names = ["setup", "loads", "init", "mul", "sepcol", "dmul", "normalize", "sepdis", "marg", "-"]
vals = list(c.values())
tot = sum(vals)
print(f"kernel {jt.last_kernel_ms():.3f} ms (profiled); total stamped cycles {tot:.3e} "
      f"= {tot / ((n + 63) // 64):.0f} per 64-case block")
for k, v in zip(names, vals):
    if v:
        print(f"   {k:10s} {v:14.3e}  {100 * v / tot:5.1f}%  {v / ((n + 63) // 64):10.0f} cyc/block")
