"""Specialized ALARM kernel (variant 3) under code-generation settings that are read from the
environment when the kernel is generated (FBN_JT_MIN_WAVES, FBN_JT_REG_ENTRIES,
FBN_JT_PREFETCH_BUDGET): one child process per setting (prebuild the code objects first with
tools/prebuild_env.py), median kernel time over interleaved repetitions.
usage: jt_env_sweep.py 'VAR=v,VAR2=w:wpc' ...   (wpc = persistent waves per CU, 0 = default)"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(wpc):
    import numpy as np
    import torch
    sys.path.insert(0, REPO)
    import fastbn_amd as F
    from fastbn_amd import synth
    xml = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
    n = 100000
    ev = synth.evidence_cases(synth.read_xmlbif(xml), n, 7, seed=1)
    jt = F.JunctionTree(F.Network(xml), device=0)
    jt.set_variant(3)
    jt.set_waves_per_cu(wpc)
    jt.set_evidence_check(False)
    d_ev = torch.from_numpy(ev).cuda()
    d_lab = torch.empty(n, dtype=torch.int32, device="cuda")
    d_marg = torch.empty((n, jt.info["sum_dom"]), dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    ms = []
    for _ in range(20):
        jt.run_device(d_ev.data_ptr(), n, d_lab.data_ptr(), d_marg.data_ptr(), s)
        ms.append(jt.last_kernel_ms())
    # parity of the last run's first 256 cases against the oracle (labels, max relative error)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    torch.cuda.synchronize()
    olab, omarg = O.OracleJT(xml).infer(ev[:256])
    lab, marg = d_lab[:256].cpu().numpy(), d_marg[:256].cpu().numpy()
    err = float(np.max(np.abs(marg - omarg) / np.maximum(np.abs(omarg), 1e-300)))
    print(json.dumps({"ms": float(np.median(ms[3:])), "min": float(min(ms)), "labels_equal": bool((lab == olab).all()),
                      "max_rel_err": err, "flagged": jt.debug_flagged_blocks()}))


if __name__ == "__main__":
    if os.environ.get("_JES_CHILD"):
        child(int(os.environ["_JES_WPC"]))
        sys.exit(0)
    for spec in sys.argv[1:]:
        envs, wpc = spec.rsplit(":", 1)
        env = dict(os.environ, _JES_CHILD="1", _JES_WPC=wpc)
        for kv in filter(None, envs.split(",")):
            k, v = kv.split("=")
            env[k] = v
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:]
        print(f"{spec:50s} {line}", flush=True)
