"""Median kernel time of the Munin-like JT batch (125k cases, 208 evidence vars, native generator):
munin_time.py [ncases] [reps] -- for A/B runs of build / environment switches, one process each."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
path = "/tmp/munin_like_time.xml"
synth.random_network(1041, seed=1041, window=12, path=path, name="munin_like")
net = F.Network(path)
ev = net.evidence_cases(n, 208, 20250131)
jt = F.JunctionTree(net, device=0)
if os.environ.get("FBN_WPC"):  # waves per CU of the launch (tuning)
    jt.set_waves_per_cu(int(os.environ["FBN_WPC"]))
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
jt.validate_device(d_ev.data_ptr(), n, None)
jt.set_evidence_check(False)
jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
torch.cuda.synchronize()
lab0 = d_lab.clone()
ms = []
for _ in range(reps):
    jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
    ms.append(jt.last_kernel_ms())
torch.cuda.synchronize()
knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("FBN_JT_") or k == "FBN_WPC")
print(f"[{knobs}] visits={jt.info['tiled_entry_visits']}: kernel ms {np.median(ms):.1f} ({' '.join(f'{m:.1f}' for m in ms)}), "
      f"labels stable {bool(torch.equal(lab0, d_lab))} labels-sum {int(d_lab.long().sum())} "
      f"marg-sum {float(d_marg.sum()):.12f} flagged {jt.info.get('flagged_blocks', 'n/a')}", flush=True)
