"""Diagnostic: repeated PC-stable runs on the config-5 dataset (1000 vars x 100k samples, levels
0-5) with per-run driver/kernel times; FBN_PC_TIMING=1 adds per-level host phase times."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
path = "/tmp/pc_c5.xml"
synth.random_network(1000, seed=1000, window=50, parent_probs=(1, 1, 1), dom=(2, 4), path=path, k_min=0)
cols = synth.forward_sample(synth.read_xmlbif(path), 100000, seed=1000)
dims = (cols.max(axis=1).astype(np.int32) + 1)
ds = F.Dataset(columns=cols, dims=dims)
ci = F.IndependenceTest(ds)  # column store resident across runs (as bench.py)
walls, drivers = [], []
for r in range(runs):
    pc = F.PCStable(0.05, 6)
    t0 = time.time()
    pc.StructLearnCompData(ci)
    wall = time.time() - t0
    walls.append(wall)
    drivers.append(pc.total_s)
    print(f"run {r}: wall {wall * 1e3:.2f} ms, driver {pc.total_s * 1e3:.2f} ms, kernels {pc.kernel_s * 1e3:.2f} ms, "
          f"tests {pc.tests_per_level.tolist()} launched {pc.launched_per_level.tolist()} edges {len(pc.edges)}",
          file=sys.stderr, flush=True)
if runs > 2:
    print(f"median over runs 2..: wall {np.median(walls[2:]) * 1e3:.3f} ms, driver {np.median(drivers[2:]) * 1e3:.3f} ms",
          file=sys.stderr, flush=True)
