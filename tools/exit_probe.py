"""Exit-path probe of the PC path (processes that ran the device-resident search
aborted with SIGSEGV inside exit() after rocprofv3's finalization).  Runs ALARM-5000 PC-stable calls
like tools/pc_once.py, then writes this process's memory map to <out>/exit_maps_<pid>.txt from an
atexit hook (registered after fastbn_amd's own, so it runs first), so that the frames of a crash
report can be symbolized against the libraries mapped at exit (tools/symbolize_crash.py).
FBN_EXIT_NO_CLOSE=1 unregisters fastbn_amd's atexit teardown (the round-4 behaviour: handles are
left to the interpreter's finalization).
usage: python tools/exit_probe.py <outdir> [calls]"""
import atexit
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import fastbn_amd as F  # noqa: E402
from fastbn_amd import api  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "."
os.makedirs(out, exist_ok=True)
if os.environ.get("FBN_EXIT_NO_CLOSE") == "1":
    atexit.unregister(api.close_all)


def dump_maps():
    with open("/proc/self/maps") as f, open(os.path.join(out, "exit_maps_%d.txt" % os.getpid()), "w") as g:
        g.write(f.read())


atexit.register(dump_maps)
ds = F.Dataset(os.path.join(REPO, "tests", "golden", "alarm", "alarm_s5000.txt"))
ci = F.IndependenceTest(ds)
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    pc = F.PCStable(0.05, 1000).StructLearnCompData(ci)
print("ok", pc.path, pc.num_ci_test, os.getpid(), flush=True)
