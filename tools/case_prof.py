"""Per-phase cycle totals of the per-case JT kernel (variant 5) on the Munin-like tree:
case_prof.py [ncases] [waves]  (FBN_JT_CDEBUG=8: s_memtime per phase, summed over waves)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
w = int(sys.argv[2]) if len(sys.argv) > 2 else 12
path = "/tmp/munin_like_prof.xml"
synth.random_network(1041, seed=1041, window=12, path=path, name="munin_like")
ev = synth.evidence_cases(synth.read_xmlbif(path), n, 208, seed=20250131)
jt = F.JunctionTree(F.Network(path), device=0)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
jt.set_variant(5)
jt.set_waves_per_cu(w)
os.environ["FBN_JT_CDEBUG"] = "8"
jt.op_cycles(True, read=False)
jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
torch.cuda.synchronize()
cyc = list(jt.op_cycles(True).values())
names = ["case set-up", "Collect set-up", "Collect decode", "Collect records", "Collect entries",
         "Distribute set-up", "Distribute decode", "Distribute records", "Distribute entries", "finishing"]
tot = sum(cyc)
print(f"kernel {jt.last_kernel_ms():.1f} ms, {n} cases, {w} waves/CU; wave-cycles per case by phase:")
for nm, c in zip(names, cyc):
    print(f"  {nm:20s} {c / n:12.0f}  {100 * c / tot:5.1f} %")
