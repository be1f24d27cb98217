"""ALARM JT kernel time vs case count (one launch per size; median of 20 after 5 warm-up): the
block latency L (16,384 cases = 256 blocks, one wave per CU), one full round (65,536 cases = 1,024
blocks, one wave per SIMD) and the 2-round headline (100,000 cases)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fastbn_amd as F  # noqa: E402

net = F.Network(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "alarm", "alarm.xml"))
dev = torch.device("cuda", 0)
N = 100000
ev = net.evidence_cases(N, 7, 20250131)
d_ev = torch.from_numpy(ev).to(dev)
d_lab = torch.empty(N, dtype=torch.int32, device=dev)
jt = F.JunctionTree(net, device=0)
d_marg = torch.empty((N, jt.info["sum_dom"]), dtype=torch.float64, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
jt.set_evidence_check(False)
for var in [int(v) for v in (sys.argv[1:] or ["3"])]:
    jt.set_variant(var)
    for n in [100000, 65536, 34464, 16384, 4096]:
        ts = []
        for i in range(25):
            jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), s)
            torch.cuda.synchronize()
            if i >= 5:
                ts.append(jt.last_kernel_ms())
        ts.sort()
        print(f"variant {var} n {n}: median {ts[len(ts) // 2]:.4f} ms min {ts[0]:.4f}", flush=True)
