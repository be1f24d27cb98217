"""Tiled JT kernel (variant 5) on the GPU: parity against the oracle on ALARM and the Munin-like
network, Munin-like timing (125k cases) and per-phase cycles, for a sweep of the LDS factor budget
(FBN_JT_TLDS, per process), waves per CU and waves per workgroup (FBN_JT_TW).
Usage: python tools/tile_probe.py [cases] [tlds:wpc[:tw] ...]"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
PHASES = ["stage", "entries/lds", "entries/global", "entries/mixed", "post sweep", "marginals", "all", "pass total"]


def child(cases, wpcs, with_v4):
    import torch
    import fastbn_amd as F
    import oracle as O
    from fastbn_amd import synth
    xml = "/tmp/munin_like.xml"
    if not os.path.exists(xml):
        synth.random_network(1041, seed=1041, window=12, path=xml, name="munin_like")
    net = F.Network(xml)
    jt = F.JunctionTree(net, device=0)
    info = {k: v for k, v in jt.info.items() if k.startswith("tiled")}
    ev = net.evidence_cases(cases, 208, 20250131)
    olab, omarg = O.OracleJT(xml).infer(ev[:16])
    dev = torch.device("cuda", 0)
    d_ev = torch.from_numpy(ev).to(dev)
    d_lab = torch.empty(cases, dtype=torch.int32, device=dev)
    d_marg = torch.empty((cases, jt.info["sum_dom"]), dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    jt.validate_device(d_ev.data_ptr(), cases, s)
    jt.set_evidence_check(False)
    runs = [(5, w) for w in wpcs] + ([(4, 0)] if with_v4 else [])
    for v, w in runs:
        jt.set_variant(v)
        jt.set_waves_per_cu(w)
        ms = []
        for _ in range(3):
            jt.run_device(d_ev.data_ptr(), cases, d_lab.data_ptr(), d_marg.data_ptr(), s)
            ms.append(jt.last_kernel_ms())
        torch.cuda.synchronize(dev)
        gm = d_marg[:16].cpu().numpy()
        rel = float(np.max(np.abs(gm - omarg) / np.maximum(np.abs(omarg), 1e-300)))
        ok = bool((d_lab[:16].cpu().numpy() == olab).all())
        line = (f"TLDS {os.environ.get('FBN_JT_TLDS', 'default')} TW {os.environ.get('FBN_JT_TW', 'default')} "
                f"v{v} wpc {w}: kernel ms "
                f"{min(ms):.1f} -> {cases / (min(ms) * 1e-3):.4g} cases/s; labels equal {ok} max rel {rel:.2e}")
        if v == 5:
            buf = (ctypes.c_ulonglong * 10)()
            F.lib.fbn_jt_debug_op_cycles(jt._h, 1, None)
            jt.run_device(d_ev.data_ptr(), cases, d_lab.data_ptr(), d_marg.data_ptr(), s)
            torch.cuda.synchronize(dev)
            F.lib.fbn_jt_debug_op_cycles(jt._h, 0, buf)
            tot = max(1, buf[6])
            line += " | " + " ".join(f"{n} {100.0 * buf[k] / tot:.1f}%" for k, n in enumerate(PHASES) if k != 6)
            line += f" | lds/wave {info['tiled_lds_bytes']}"
        print(line, flush=True)


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000
    if os.environ.get("_TP_CHILD"):
        child(cases, [int(w) for w in os.environ["_TP_WPC"].split(",")], os.environ.get("_TP_V4") == "1")
        return
    import fastbn_amd as F
    import oracle as O
    from fastbn_amd import synth
    alarm = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
    jt = F.JunctionTree(F.Network(alarm), device=0)
    jt.set_variant(5)
    ev = synth.evidence_cases(synth.read_xmlbif(alarm), 1000, 7, seed=11)
    lab, marg = jt.infer(ev)
    olab, omarg = O.OracleJT(alarm).infer(ev)
    rel = np.max(np.abs(marg - omarg) / np.maximum(np.abs(omarg), 1e-300))
    print(f"alarm v5: labels equal {bool((lab == olab).all())} max rel {rel:.3e}", flush=True)
    specs = sys.argv[2:] or ["16384:8", "8192:16,12", "32768:4"]
    for i, sp in enumerate(specs):
        tl, w, *tw = sp.split(":")  # LDS factor bytes per workgroup : waves per CU [: waves per workgroup]
        env = dict(os.environ, _TP_CHILD="1", FBN_JT_TLDS=tl, _TP_WPC=w, _TP_V4="1" if i == 0 else "0")
        if tw:
            env["FBN_JT_TW"] = tw[0]
        subprocess.run([sys.executable, __file__, str(cases)], check=True, env=env)


if __name__ == "__main__":
    main()
