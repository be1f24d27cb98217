"""Diagnostic: config-5 skeleton after level 0 -> degree statistics and the level-1 candidate-set
count (every edge's |adj(x)| - 1 + |adj(y)| - 1), and the triple-Gram size sum_x (d_x-1) R_x^2."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

cols, dims = synth.config5_dataset()
pc = F.PCStable(0.05, 1).StructLearnCompData(F.IndependenceTest(F.Dataset(columns=cols, dims=dims)))
n = len(dims)
adj = [[] for _ in range(n)]
for a, b in pc.edges:
    adj[a].append(b)
    adj[b].append(a)
deg = np.array([len(a) for a in adj])
cands = sum(deg[a] - 1 + deg[b] - 1 for a, b in pc.edges)
R = np.array([sum(dims[v] - 1 for v in adj[x]) for x in range(n)])
gram = int(sum((dims[x] - 1) * R[x] ** 2 for x in range(n)))
print(f"edges {len(pc.edges)} deg mean {deg.mean():.1f} max {deg.max()} cands {cands} "
      f"R mean {R.mean():.1f} max {R.max()} gram ints {gram} ({gram * 4 / 2**20:.1f} MiB) "
      f"gram popc-words {int(sum((dims[x] - 1) * R[x] * (R[x] + 1) // 2 for x in range(n))) * 3128}")
