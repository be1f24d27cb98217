"""ALARM headline step as bench.py times it (100k cases, back-to-back steps on one stream, torch
events around each step, wall clock over the steps): ms per step and event ms per step, for
comparing launch-level variants (e.g. FBN_JT_NO_FIXUP=1, diagnostic).  alarm_step_probe.py [steps] [timing 0/1]"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ktiming = int(sys.argv[2]) if len(sys.argv) > 2 else 1
xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
n = 100000
ev = synth.evidence_cases(synth.read_xmlbif(xml), n, 7, seed=1)
jt = F.JunctionTree(F.Network(xml), device=0)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream()
jt.validate_device(d_ev.data_ptr(), n, s.cuda_stream)
jt.set_evidence_check(False)
jt.set_kernel_timing(bool(ktiming))
for _ in range(5):
    jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), s.cuda_stream)
torch.cuda.synchronize()
for rep in range(3):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    kms = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        evs[i][0].record(s)
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), s.cuda_stream)
        evs[i][1].record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    ev_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    kms = jt.last_kernel_ms() if ktiming else float("nan")
    print(f"rep {rep}: ms/step {wall:.4f}  event ms {ev_ms:.4f}  last_kernel_ms {kms:.4f}  "
          f"flagged {jt.debug_flagged_blocks()}", flush=True)
