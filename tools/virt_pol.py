"""Diagnostic: streamed JT kernel (variant 4) on the Munin-like network under the scratch-table
cache policies of jt_virt.hip (FBN_JT_VPOL 0..3).  Results stay exact; only the timing changes."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = sys.argv[1] if len(sys.argv) > 1 else "125000"
for pol in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,3").split(","):
    env = dict(os.environ, FBN_JT_VPOL=pol)
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "munin_probe.py"), n, "4"], env=env,
                         capture_output=True, text=True, timeout=300).stdout
    line = [l for l in out.split("\n") if l.startswith("variant")]
    print(f"pol={pol}: {line[0] if line else out[-300:]}", flush=True)
