"""PC-stable on the synthetic SURVEY §8(d) config 5 dataset (1000 vars x 100k samples: node i draws
k ~ U{0..2} parents from the previous 50, domains U{2..4}, Dirichlet(1) CPTs, seed 1000).
pc_probe.py [nvars] [nsamples] [depth]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

nv = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
ns = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
t0 = time.time()
path = "/tmp/pc_c5.xml"
synth.random_network(nv, seed=1000, window=50, parent_probs=(1, 1, 1), dom=(2, 4), path=path, k_min=0)
cols = synth.forward_sample(synth.read_xmlbif(path), ns, seed=1000)
dims = (cols.max(axis=1).astype(np.int32) + 1)
print(f"dataset {nv} x {ns} generated in {time.time() - t0:.1f} s", flush=True)
ds = F.Dataset(columns=cols, dims=dims)
pc = F.PCStable(0.05, depth)
t0 = time.time()
pc.StructLearnCompData(ds)
wall = time.time() - t0
print(f"depth {depth}: tests/level {pc.tests_per_level.tolist()} launched {pc.launched_per_level.tolist()}")
print(f"wall {wall:.3f} s (driver {pc.total_s:.3f} s, kernels {pc.kernel_s:.3f} s): "
      f"{pc.num_ci_test / pc.total_s:.0f} CI-tests/s, {len(pc.edges)} edges", flush=True)
