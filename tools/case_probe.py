"""Munin-like JT: variant 4 (streamed) vs variant 5 (per-case) timing and agreement on one GPU.
case_probe.py [ncases] [variants, e.g. 4,5] [waves for 5]"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
variants = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "4,5").split(",")]
waves = [int(w) for w in (sys.argv[3] if len(sys.argv) > 3 else "0").split(",")]
dbgs = [int(w) for w in (sys.argv[4] if len(sys.argv) > 4 else "0").split(",")]  # variant-5 ablations
path = "/tmp/munin_like_probe.xml"
synth.random_network(1041, seed=1041, window=12, path=path, name="munin_like")
ev = synth.evidence_cases(synth.read_xmlbif(path), n, 208, seed=20250131)
jt = F.JunctionTree(F.Network(path), device=0)
d_ev = torch.from_numpy(ev).cuda()
d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
jt.validate_device(d_ev.data_ptr(), n, None)
jt.set_evidence_check(False)
ref = None
for v, w, dbg in [(v, w, d) for v in variants for w in (waves if v == 5 else [0]) for d in (dbgs if v == 5 else [0])]:
    if dbg:
        os.environ["FBN_JT_CDEBUG"] = str(dbg)  # ablation: no fixup pass, wrong results
    else:
        os.environ.pop("FBN_JT_CDEBUG", None)
    if True:
        jt.set_variant(v)
        jt.set_waves_per_cu(w)
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), None)
            torch.cuda.synchronize()
            ts.append(jt.last_kernel_ms())
        lab, marg = d_lab.cpu().numpy(), d_marg.cpu().numpy()
        msg = ""
        if dbg:
            pass
        elif ref is None:
            ref = (lab, marg)
        else:
            rel = np.abs(marg - ref[1]) / np.maximum(np.abs(ref[1]), 1e-300)
            msg = f"labels equal {np.mean(lab == ref[0]):.6f}, max rel {rel.max():.3g}"
        ms = float(np.median(ts))
        print(f"variant {v} waves {w} dbg {dbg}: {ms:.2f} ms / {n} cases = {n / ms * 1e3:.4g} cases/s {msg}", flush=True)
