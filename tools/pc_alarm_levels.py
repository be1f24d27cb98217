"""Diagnostic: PC-stable on alarm_s5000 repeated; per-run driver / kernel ms and launched tests.
Combine with FBN_PC_TIMING=1 (per-level host phases) or FBN_CI_FORCE_BITS=1 (bit-sliced kernel)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ds = F.Dataset(os.path.join(REPO, "tests/golden/alarm/alarm_s5000.txt"))
ci = F.IndependenceTest(ds)
pc = F.PCStable(0.05, 1000)
for _ in range(runs):
    pc.StructLearnCompData(ci)
    print(f"driver {pc.total_s * 1e3:.3f} ms, kernels {pc.kernel_s * 1e3:.3f} ms, launched "
          f"{pc.launched_per_level.tolist()}, edges {len(pc.edges)}, SHD {pc.GetSHD(os.path.join(REPO, 'tests/golden/alarm/alarm.bif'))}",
          flush=True)
