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


def test_cli_rccl_path_at_one_gpu():
    """--gpus path of the C++ host (cli/MultiGpu.h: ncclCommInitAll, one thread per GPU) forced on
    the box's one GPU (FBN_PC_DIST_FORCE_EXCHANGE): PC through ncclBroadcast of the columns + the
    native session with ncclAllGather of the records and pair tables; JT cases through
    fbn_jt_run_device, scored on the device (fbn_jt_score_terms_device) + all-gathers of the labels
    and the per-case terms -- the same result lines as the one-GPU path."""
    env = dict(os.environ, FBN_PC_DIST_FORCE_EXCHANGE="1")

    def run_env(args):
        out = subprocess.run([CLI] + args + ["--gpus", "1", "--prefix", GOLD + "/"], capture_output=True, text=True,
                             timeout=300, env=env)
        assert out.returncode == 0, out.stderr
        return out.stdout

    pc = run_env(["-a", "0", "-f1", "alarm/alarm.bif", "-f2", "alarm/alarm_s5000.txt"])
    # ALARM-5000 is a small graph: replicas of the one-launch search + ncclBroadcast of rank 0's record
    assert "(RCCL, replicas" in pc and "# of CI-tests is 5206" in pc and "SHD = 5" in pc, pc
    plain = run(["-a", "0", "-f1", "alarm/alarm.bif", "-f2", "alarm/alarm_s5000.txt"])
    pick = lambda s: [ln for ln in s.splitlines() if ln.startswith(("Level", "# of CI", "# remaining", "SHD"))]
    assert pick(pc) == pick(plain)
    # the edge-split session (larger graphs) on the same data: FBN_PC_NO_SMALL makes it ineligible
    env["FBN_PC_NO_SMALL"] = "1"
    split = run_env(["-a", "0", "-f1", "alarm/alarm.bif", "-f2", "alarm/alarm_s5000.txt"])
    del env["FBN_PC_NO_SMALL"]
    assert "(RCCL, edges split" in split and pick(split) == pick(plain), split
    jt_args = ["-a", "2", "-f0", "alarm/alarm.xml", "-f3", "alarm/testing_alarm_1k_p20", "-f4", "alarm/alarm_1k_pt"]
    jt = run_env(jt_args)
    assert "(RCCL" in jt and re.search(r"accuracy = 1\b", jt), jt
    jplain = run(jt_args)
    pickj = lambda s: [ln for ln in s.splitlines() if ln.startswith(("average", "accuracy"))]
    assert pickj(jt) == pickj(jplain)


def test_cli_gpus_beyond_visible_devices_fails_cleanly():
    out = subprocess.run([CLI, "-a", "0", "--gpus", "64", "--prefix", GOLD + "/"], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode != 0 and "HIP device(s) visible" in out.stderr
