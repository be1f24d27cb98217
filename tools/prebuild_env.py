"""Prebuild the ALARM specialized kernel under tuning env settings: prebuild_env.py 'VAR=v,VAR2=w' ..."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
procs = []
for spec in sys.argv[1:]:
    env = dict(os.environ)
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        env[k] = v
    code = ("import sys; sys.path.insert(0, %r); import fastbn_amd as f; "
            "jt = f.JunctionTree(f.Network(%r), device=-1); print(%r, jt.build_kernel())"
            % (REPO, os.path.join(REPO, "tests/golden/alarm/alarm.xml"), spec))
    procs.append(subprocess.Popen([sys.executable, "-c", code], env=env))
sys.exit(max(p.wait() for p in procs))
