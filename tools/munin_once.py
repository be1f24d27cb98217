"""One Munin-like JT launch for rocprofv3 PMC passes: munin_once.py [ncases] [variant] [waves]."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
variant = int(sys.argv[2]) if len(sys.argv) > 2 else -1
waves = int(sys.argv[3]) if len(sys.argv) > 3 else 0
path = "/tmp/munin_like_once.xml"
synth.random_network(1041, seed=1041, window=12, path=path, name="munin_like")
ev = synth.evidence_cases(synth.read_xmlbif(path), n, 208, seed=20250131)
jt = F.JunctionTree(F.Network(path), device=0)
jt.set_variant(variant)
jt.set_waves_per_cu(waves)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
torch.cuda.synchronize()
print("ok", jt.last_kernel_ms(), jt.refresh_info()["variant"])
