"""Run the JT kernel a few times (for rocprofv3 PMC passes): jt_once.py [variant] [waves] [reps] [cases] [layout]
(layout 1: variable-major marginals, fbn_jt_set_output_layout)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
waves = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
n = int(sys.argv[4]) if len(sys.argv) > 4 else 100000
ev = synth.evidence_cases(synth.read_xmlbif(xml), n, 7, seed=1)
jt = F.JunctionTree(F.Network(xml), device=0)
jt.set_variant(variant)
jt.set_waves_per_cu(waves)
layout = int(sys.argv[5]) if len(sys.argv) > 5 else 0
jt.set_output_layout(layout)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
for _ in range(reps):
    jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
torch.cuda.synchronize()
print("ok", jt.last_kernel_ms())
