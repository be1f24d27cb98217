"""Per-phase wave-cycles of the tiled kernel (variant 5) on the Munin-like tree, with the plan's step
counts and cycles per step: tile_phase.py [ncases].  Plan knobs (FBN_JT_*) per process."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import fastbn_amd as F  # noqa: E402
import tile_emulator as TE  # noqa: E402
from fastbn_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32000
path = "/tmp/munin_like_phase.xml"
synth.random_network(1041, seed=1041, window=12, path=path, name="munin_like")
net = F.Network(path)
ev = net.evidence_cases(n, 208, 20250131)
jt = F.JunctionTree(net, device=0)
passes, tab, _, _ = jt.tile_program()
steps = np.zeros(8)
for prow in passes:
    P = dict(zip(TE.F, (int(x) for x in prow)))
    k = 1 if P["nl"] == P["nf"] else 2 if P["nl"] == 0 else 3
    steps[k] += P["rounds"] * P["nRo"] * P["nRi"]
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
plain = []
for _ in range(3):
    jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
    plain.append(jt.last_kernel_ms())
jt.op_cycles(True, read=False)
jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
torch.cuda.synchronize()
cyc = np.array(list(jt.op_cycles(False).values())[:7], dtype=np.float64)
names = ["staging", "entries LDS", "entries global", "entries mixed", "totals/post", "marginals", "all"]
groups = (n + 15) // 16
knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("FBN_JT_"))
print(f"[{knobs}] kernel {np.median(plain):.1f} ms (profiled "
      f"{jt.last_kernel_ms():.1f}), {n} cases; wave-cycles per case group:")
for k, nm in enumerate(names):
    extra = f"  steps {steps[k]:8.0f}  cyc/step {cyc[k] / groups / steps[k]:8.1f}" if steps[k] else ""
    print(f"  {nm:18s} {cyc[k] / groups:14.0f}  {100 * cyc[k] / cyc[6]:5.1f} %{extra}")
