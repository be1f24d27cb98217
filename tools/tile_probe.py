"""Tiled JT kernel (variant 5) on the GPU: parity against the oracle on ALARM and the Munin-like
network, then Munin-like timing of variants 5 and 4 (125k cases).  Usage: python tools/tile_probe.py [cases]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    import torch
    import fastbn_amd as F
    import oracle as O
    from fastbn_amd import synth
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000
    alarm = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
    jt = F.JunctionTree(F.Network(alarm), device=0)
    jt.set_variant(5)
    ev = synth.evidence_cases(synth.read_xmlbif(alarm), 1000, 7, seed=11)
    lab, marg = jt.infer(ev)
    olab, omarg = O.OracleJT(alarm).infer(ev)
    rel = np.max(np.abs(marg - omarg) / np.maximum(np.abs(omarg), 1e-300))
    print(f"alarm v5: labels equal {bool((lab == olab).all())} max rel {rel:.3e}", flush=True)
    xml = "/tmp/munin_like.xml"
    synth.random_network(1041, seed=1041, window=12, path=xml, name="munin_like")
    t0 = time.time()
    net = F.Network(xml)
    jt = F.JunctionTree(net, device=0)
    print(f"munin plan {time.time() - t0:.2f} s, tiled info",
          {k: v for k, v in jt.info.items() if k.startswith("tiled")}, flush=True)
    ev = net.evidence_cases(cases, 208, 20250131)
    olab, omarg = O.OracleJT(xml).infer(ev[:16])
    dev = torch.device("cuda", 0)
    d_ev = torch.from_numpy(ev).to(dev)
    d_lab = torch.empty(cases, dtype=torch.int32, device=dev)
    d_marg = torch.empty((cases, jt.info["sum_dom"]), dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    jt.validate_device(d_ev.data_ptr(), cases, s)
    jt.set_evidence_check(False)
    for v in (5, 4):
        jt.set_variant(v)
        ms = []
        for _ in range(3):
            jt.run_device(d_ev.data_ptr(), cases, d_lab.data_ptr(), d_marg.data_ptr(), s)
            ms.append(jt.last_kernel_ms())
        torch.cuda.synchronize(dev)
        gm = d_marg[:16].cpu().numpy()
        rel = float(np.max(np.abs(gm - omarg) / np.maximum(np.abs(omarg), 1e-300)))
        ok = bool((d_lab[:16].cpu().numpy() == olab).all())
        print(f"munin v{v}: kernel ms {ms} -> {cases / (min(ms) * 1e-3):.4g} cases/s; labels equal {ok} "
              f"max rel {rel:.3e}", flush=True)


if __name__ == "__main__":
    main()
