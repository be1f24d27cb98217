"""bench.py's full-batch JT checks on CPU tensors: the oracle's own ALARM outputs pass
`jt_full_batch_properties`, and a corrupted label / marginal row / evidence row is caught."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import bench  # noqa: E402
import oracle as O  # noqa: E402
from fastbn_amd import synth  # noqa: E402

ALARM = os.path.join(REPO, "tests", "golden", "alarm", "alarm.xml")


def _batch(n=300, evid=7, seed=5):
    import torch
    ev = synth.evidence_cases(synth.read_xmlbif(ALARM), n, evid, seed=seed)
    ev[::3, 0] = -1  # variable 0 (the label) free in most cases, observed in some
    lab, marg = O.OracleJT(ALARM).infer(ev)
    o = O.OracleJT(ALARM)
    return torch.from_numpy(ev), torch.from_numpy(lab), torch.from_numpy(marg), o.dims


def test_oracle_outputs_pass():
    ev, lab, marg, dims = _batch()
    p = bench.jt_full_batch_properties(ev, lab, marg, dims, chunk=128)
    assert p["ok"] and p["cases"] == 300 and p["label_mismatches"] == 0
    assert p["max_abs_row_sum_err"] <= 1e-12


def test_corruptions_are_caught():
    ev, lab, marg, dims = _batch()
    free = int(np.flatnonzero(ev[:, 0].numpy() < 0)[0])
    d0 = int(dims[0])
    bad = lab.clone()
    m0 = marg[free, :d0]
    bad[free] = int(np.argsort(m0.numpy())[0])  # the smallest state instead of the largest
    assert not bench.jt_full_batch_properties(ev, bad, marg, dims)["ok"]
    m = marg.clone()
    m[free, :d0] *= 1.001  # a row that no longer sums to 1
    p = bench.jt_full_batch_properties(ev, lab, m, dims)
    assert not p["ok"] and p["max_abs_row_sum_err"] > 1e-6
    m = marg.clone()
    obs = np.argwhere(ev.numpy() >= 0)[0]
    off = int(np.concatenate([[0], np.cumsum(dims)])[obs[1]])
    m[obs[0], off] = 0.5  # an evidence variable's row must stay zero
    p = bench.jt_full_batch_properties(ev, lab, m, dims)
    assert not p["ok"] and not p["evidence_rows_zero"]


def test_oracle_sample_indices():
    s = bench.oracle_sample(100_000, 256, 1792)
    assert s[0] == 0 and s[-1] == 99_999 and len(s) == len(np.unique(s)) and (np.diff(s) > 0).all()
    assert set(range(256)) <= set(s.tolist())
    assert list(bench.oracle_sample(5, 16, 48)) == [0, 1, 2, 3, 4]


def _bench(args, env_extra=None):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       env=env, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def test_bench_gpus_2_launches_two_ranks():
    """`bench.py --gpus 2` without a launcher starts two rank processes itself (torch.distributed.run,
    gloo here: --launcher-check runs the rank plumbing only) and rank 0 reports world size 2."""
    rc, line, err = _bench(["--gpus", "2", "--launcher-check"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2 and line["world_size_seen"] == 2 and line["ranks_seen"] == [0, 1]


def test_bench_gpus_1_stays_one_process():
    rc, line, err = _bench(["--launcher-check"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 1 and line["world_size_seen"] == 1 and line["ranks_seen"] == [0]


def test_bench_rejects_gpus_world_size_mismatch():
    rc, line, err = _bench(["--gpus", "2", "--launcher-check"], {"WORLD_SIZE": "3", "RANK": "0"})
    assert rc == 2 and line is None and "WORLD_SIZE=3" in err
