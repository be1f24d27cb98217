"""Diagnostic: time the streamed JT kernel (variant 4) on the Munin-like network with pass types
skipped (FBN_JT_VDEBUG bits: 1 SEPCOL, 2 SEPDIS, 4 MARG, 8 Distribute SUM, 16 whole Distribute).
Results are wrong in the ablated runs; only the timings mean something."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = sys.argv[1] if len(sys.argv) > 1 else "125000"
for dbg in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,4,8,16,31").split(","):
    env = dict(os.environ, FBN_JT_VDEBUG=dbg)
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "munin_probe.py"), n, "4"], env=env,
                         capture_output=True, text=True).stdout
    line = [l for l in out.split("\n") if l.startswith("variant")]
    print(f"dbg={dbg}: {line[0] if line else out[-300:]}", flush=True)
