"""ALARM specialized JT kernel (variant 3): time the generated kernel under register-budget settings
(FBN_JT_PREFETCH_BUDGET, FBN_JT_REG_ENTRIES), each JIT-compiled in this process, results checked
bit-identical to the default.  jt_budget_sweep.py "budget:entries,..." [cases]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

cfgs = [tuple(x.split(":")) for x in (sys.argv[1] if len(sys.argv) > 1 else "200:96,180:96,160:96,200:80").split(",")]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
ev = synth.evidence_cases(synth.read_xmlbif(xml), n, 7, seed=20250131)
d_ev = torch.from_numpy(ev).cuda()
ref = None
for budget, entries in [("", "")] + cfgs:
    for k, v in (("FBN_JT_PREFETCH_BUDGET", budget), ("FBN_JT_REG_ENTRIES", entries)):
        if v:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)
    jt = F.JunctionTree(F.Network(xml), device=0)
    d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
    d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
    jt.validate_device(d_ev.data_ptr(), n, None)
    jt.set_evidence_check(False)
    jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
    torch.cuda.synchronize()
    ts = []
    for _ in range(15):
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
        torch.cuda.synchronize()
        ts.append(jt.last_kernel_ms())
    lab, marg = d_lab.cpu().numpy(), d_marg.cpu().numpy()
    same = "ref" if ref is None else bool((lab == ref[0]).all() and (marg == ref[1]).all())
    if ref is None:
        ref = (lab, marg)
    print(f"budget {budget or 'default'} entries {entries or 'default'}: variant {jt.refresh_info()['variant']} "
          f"median {np.median(ts):.4f} ms min {np.min(ts):.4f} ms, identical {same}", flush=True)
