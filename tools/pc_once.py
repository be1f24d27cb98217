"""One ALARM-5000 PC-stable call (the device-resident search, pc_small_kernel) for rocprofv3 PMC passes."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402

ds = F.Dataset(os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt"))
ci = F.IndependenceTest(ds)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    pc = F.PCStable(0.05, 1000).StructLearnCompData(ci)
print("ok", pc.path, pc.num_ci_test, flush=True)
