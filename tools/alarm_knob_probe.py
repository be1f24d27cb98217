"""The ALARM headline kernel (variable-major marginals, 100k cases) under this process's FBN_JT_*
codegen knobs: ms per 100k over K runs on the launch stream, median of rounds.  One process per
setting (the plan reads the knobs when it generates its kernel).  usage: alarm_knob_probe.py [steps] [rounds]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
n = 100_000
net = F.Network(xml)
ev = net.evidence_cases(n, 7, 20250131)
jt = F.JunctionTree(net, device=0)
if os.environ.get("FBN_WPC"):
    jt.set_waves_per_cu(int(os.environ["FBN_WPC"]))
dev = torch.device("cuda", 0)
d_ev = torch.from_numpy(ev).to(dev)
d_lab = torch.empty(n, dtype=torch.int32, device=dev)
d_marg = torch.empty(n * jt.info["sum_dom"], dtype=torch.float64, device=dev)
st = torch.cuda.current_stream(dev)
jt.validate_device(d_ev.data_ptr(), n, st.cuda_stream)
jt.set_evidence_check(False)
jt.set_kernel_timing(False)
jt.set_output_layout(1)
res = []
for r in range(rounds):
    for _ in range(3):
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), st.cuda_stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    a.record(st)
    for _ in range(steps):
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), st.cuda_stream)
    b.record(st)
    torch.cuda.synchronize(dev)
    res.append(a.elapsed_time(b) / steps)
knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("FBN_JT_") or k == "FBN_WPC")
print(f"[{knobs}] variant {jt.refresh_info()['variant']}: ms per 100k median {np.median(res):.4f} "
      f"({' '.join(f'{x:.4f}' for x in res)})", flush=True)
