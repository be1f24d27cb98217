"""A/B of the ALARM headline kernel's output layouts (100k cases, bench.py's timing: one event pair
around K runs on the launch stream, evidence checked once): case-major vs variable-major marginals.
usage: alarm_layout_probe.py [steps] [rounds]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
n = 100_000
net = F.Network(xml)
ev = net.evidence_cases(n, 7, 20250131)
jt = F.JunctionTree(net, device=0)
dev = torch.device("cuda", 0)
d_ev = torch.from_numpy(ev).to(dev)
d_lab = torch.empty(n, dtype=torch.int32, device=dev)
d_marg = torch.empty(n * jt.info["sum_dom"], dtype=torch.float64, device=dev)
st = torch.cuda.current_stream(dev)
jt.validate_device(d_ev.data_ptr(), n, st.cuda_stream)
jt.set_evidence_check(False)
jt.set_kernel_timing(False)
res = {0: [], 1: []}
for r in range(rounds):
    for layout in (0, 1):
        jt.set_output_layout(layout)
        for _ in range(3):
            jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), st.cuda_stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        a.record(st)
        for _ in range(steps):
            jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), st.cuda_stream)
        b.record(st)
        torch.cuda.synchronize(dev)
        res[layout].append(a.elapsed_time(b) / steps)
for layout in (0, 1):
    print(f"layout {layout}: ms per 100k = {' '.join(f'{x:.4f}' for x in res[layout])}", flush=True)
