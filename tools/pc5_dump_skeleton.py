"""Diagnostic: config-5 skeleton + sepsets (device run) -> gpurun_out/c5_skel.npz, for profiling the
host orientation on a CPU (fastbn_amd.orient_skeleton)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import synth  # noqa: E402

cols, dims = synth.config5_dataset()
pc = F.PCStable(0.05, 6).StructLearnCompData(F.IndependenceTest(F.Dataset(columns=cols, dims=dims)))
sep = pc.sepset
keys = np.array(sorted(sep), np.int32).reshape(-1, 2)
lens = np.array([len(sep[tuple(k)]) for k in keys], np.int32)
vals = np.array([v for k in keys for v in sep[tuple(k)]], np.int32)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(REPO, "gpurun_out", "c5_skel.npz"), edges=np.array(pc.edges, np.int32),
                    keys=keys, lens=lens, vals=vals, oriented=np.array(pc.oriented, np.int32))
print("edges", len(pc.edges), "sepsets", len(keys))
