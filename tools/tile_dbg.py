"""Diagnostic: the tiled kernel (variant 5) on a few ALARM cases with the exact fixup disabled
(FBN_JT_NO_FIXUP=1 must be set): worst relative error per variable vs the oracle, NaN count."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import fastbn_amd as F  # noqa: E402
import oracle as O  # noqa: E402
from fastbn_amd import synth  # noqa: E402

xml = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")
n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
net = F.Network(xml)
jt = F.JunctionTree(net, device=0)
jt.set_variant(5)
ev = synth.evidence_cases(synth.read_xmlbif(xml), n, max(1, len(net.dims) // 5), seed=11)
lab, marg = jt.infer(ev)
olab, omarg = O.OracleJT(xml).infer(ev)
rel = np.abs(marg - omarg) / np.maximum(np.abs(omarg), 1e-300)
print("labels equal", bool((lab == olab).all()), "nan", int(np.isnan(marg).sum()), "max rel", float(np.nanmax(rel)))
off = np.concatenate([[0], np.cumsum(net.dims)])
bad = [(v, float(np.nanmax(rel[:, off[v]:off[v + 1]]))) for v in range(len(net.dims))]
print("worst vars", sorted(bad, key=lambda x: -x[1])[:8])
print("case 0 marg[0:8]", marg[0, :8], "oracle", omarg[0, :8])
