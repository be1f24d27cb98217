"""The level-1 information screen (ci_bits.hip `l1_plausible`) checked against the oracle's own test
log, on the CPU: every level-1 test the reference's algorithm finds INDEPENDENT passes the screen,
so the candidates the screen skips are dependent and the device's counted tests, edges and sepsets
stay the reference's (src/PCStable.cpp:465-551).  The screen's argument: with plug-in mutual
information over the same samples, I(X;Y) <= I(X;Z) + I(X;Y|Z) (chain rule), G^2 = 2N I, and an
independent test has G^2 <= the chi-square quantile of its df <= that of (dx-1)(dy-1)dz."""
import os

import numpy as np
import pytest
from conftest import ALARM

import oracle as O

ALPHA = 0.05


def _crit(df):
    from scipy.stats import chi2
    return float(chi2.isf(ALPHA, df))


def _plausible(mi, dims, n, x, y, z):
    """The device predicate (ci_bits.hip l1_plausible) with the chi-square quantile for the band's hi."""
    df = (dims[x] - 1) * (dims[y] - 1) * dims[z]
    if df <= 0:
        return True
    lim = mi[x, y] - (_crit(df) * (1 + 1e-9) / (2 * n) + 1e-9)
    return lim <= 0 or (mi[x, z] >= lim and mi[y, z] >= lim)


def _check(od, n):
    r = od.pc_stable(ALPHA, 1000, 1, keep_log=True)
    V = len(od.dims)
    mi = np.zeros((V, V))
    level1 = []
    for lvl, x, y, z, g2, df, p, ind in r["log"]:
        if lvl == 0:
            mi[x, y] = mi[y, x] = g2 / (2 * n)
        elif lvl == 1:
            level1.append((x, y, z[0], ind))
    assert level1, "no level-1 tests"
    skipped = 0
    for x, y, z, ind in level1:
        ok = _plausible(mi, od.dims, n, x, y, z)
        if ind:
            assert ok, f"independent test ({x}, {y} | {z}) screened out"
        skipped += not ok
    return len(level1), skipped


def test_screen_keeps_every_independent_test_alarm5000():
    od = O.OracleDataset(csv=os.path.join(ALARM, "alarm_s5000.txt"))
    total, skipped = _check(od, 5000)
    assert skipped > 0  # the screen does remove work on ALARM-5000's level 1


@pytest.mark.parametrize("nvars,ns", [(120, 20000)])
def test_screen_keeps_every_independent_test_config5_like(nvars, ns):
    """The config-5 generator at a size the oracle finishes in seconds."""
    from fastbn_amd import synth
    cols, dims = synth.config5_dataset(nvars, ns)
    od = O.OracleDataset(columns=cols, dims=dims)
    total, skipped = _check(od, ns)
    assert skipped > total // 4  # most of the counted level-1 tests are decided by the screen
