"""The drop-in CLI (`fastbn_amd/BayesianNetwork -a 0|2`) end to end on the GPU: same flags and
result lines as the reference's main (src/main.cpp:17-201)."""
import os
import re
import subprocess

import pytest
from conftest import GOLD, REPO

CLI = os.path.join(REPO, "fastbn_amd", "BayesianNetwork")
pytestmark = pytest.mark.gpu


def run(args):
    out = subprocess.run([CLI] + args + ["--prefix", GOLD + "/"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    return out.stdout


def test_cli_jt_alarm():
    out = run(["-a", "2", "-f0", "alarm/alarm.xml", "-f3", "alarm/testing_alarm_1k_p20", "-f4", "alarm/alarm_1k_pt"])
    assert re.search(r"accuracy = 1\b", out), out


def test_cli_pc_alarm_shd():
    out = run(["-a", "0", "-f1", "alarm/alarm.bif", "-f2", "alarm/alarm_s5000.txt"])
    assert "# of CI-tests is 5206" in out, out
    assert "(0 decisions within 1e-9)" in out, out  # decision-margin log, SURVEY §8(c)
    assert "SHD = 5" in out, out
