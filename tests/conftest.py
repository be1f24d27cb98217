"""Shared fixtures.  `-m "not gpu"` runs here (no GPU); `-m gpu` runs on an MI355X box."""
import gzip
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
ALARM = os.path.join(GOLD, "alarm")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def read_ref_marg(path, dims):
    """Parse a reference harness .marg(.gz) dump -> (labels, marginals [n][sum dom], mse_sum, hd_sum)."""
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        lines = f.read().split("\n")
    labels, rows, i, mse, hd = [], [], 0, None, None
    V = len(dims)
    while i < len(lines):
        ln = lines[i]
        if ln.startswith("case"):
            labels.append(int(ln.split()[3]))
            row = []
            for v in range(V):
                row += [float(x) for x in lines[i + 1 + v].split()]
            rows.append(row)
            i += 1 + V
        elif ln.startswith("mse_sum"):
            t = ln.split()
            mse, hd = float(t[1]), float(t[3])
            i += 1
        else:
            i += 1
    return np.array(labels, np.int32), np.array(rows), mse, hd


def read_pt_file(path, dims, ncases):
    """alarm_1k_pt -> golden [n][sum dom] with -1 in the first slot of evidence nodes."""
    SD = int(np.sum(dims))
    out = np.zeros((ncases, SD))
    with open(path) as f:
        lines = f.read().split("\n")
    k = 0
    for c in range(ncases):
        off = 0
        for v, d in enumerate(dims):
            ln = lines[k].rstrip()
            k += 1
            if not ln:
                out[c, off] = -1
            else:
                out[c, off:off + d] = [float(x) for x in ln.split(" ")[:d]]
            off += d
    return out


def read_ci_fixture(path):
    with gzip.open(path, "rt") as f:
        lines = f.read().strip().split("\n")
    dims = [int(x) for x in lines[1].split()[1:]]
    colhash = {}
    tests = []
    for ln in lines[2:]:
        t = ln.split()
        if t[0] == "colhash":
            colhash[int(t[1])] = int(t[2])
        elif t[0] == "test":
            x, y, d = int(t[1]), int(t[2]), int(t[3])
            z = [int(v) for v in t[4:4 + d]]
            colon = t.index(":")
            counts = np.array([int(v) for v in t[colon + 1:]], np.int32)
            tests.append((x, y, z, counts))
    return dims, colhash, tests


def fnv1a(col):
    h = 1469598103934665603
    for v in col.tolist():
        h ^= v
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.fixture(scope="session")
def alarm_paths():
    return {k: os.path.join(ALARM, v) for k, v in {
        "xml": "alarm.xml", "bif": "alarm.bif", "test": "testing_alarm_1k_p20", "pt": "alarm_1k_pt",
        "csv": "alarm_s5000.txt", "rand": "rand_evidence.libsvm"}.items()}


def have_gpu():
    try:
        import fastbn_amd
        return fastbn_amd.device_count() > 0
    except Exception:
        return False
