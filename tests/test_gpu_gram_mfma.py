"""The level-0 Gram on the gfx950 matrix cores (ci_gram_mfma.hip: FP4 one-hot x FP4 MFMA, split-K
uint16 slabs) against the popcount Gram kernel (FBN_CI_GRAM_NO_MFMA) on ragged shapes: leading-row
counts that are not multiples of the 256-row tile, sample counts that are not multiples of the
128-sample stage, mixed state counts.  Every level-0 pair table (counts recorded for level 1) must be
identical, and each table must sum to N.  Config 5 itself is pinned against the reference's tables
in test_gpu_pc_c5_pinned.py (its level-0 batch runs this kernel by default)."""
import numpy as np
import pytest

import fastbn_amd as F

pytestmark = pytest.mark.gpu


def _dataset(nvars, N, seed):
    rng = np.random.default_rng(seed)
    dims = rng.integers(2, 5, nvars).astype(np.int32)
    cols = np.empty((nvars, N), np.uint8)
    base = rng.integers(0, 4, N)
    for v in range(nvars):  # mildly dependent columns: tables far from uniform
        noise = rng.integers(0, dims[v], N)
        keep = rng.random(N) < 0.3
        cols[v] = np.where(keep, base % dims[v], noise)
    return cols, dims


@pytest.mark.parametrize("nvars,N,seed", [(520, 30001, 1), (700, 20480, 2), (260, 100003, 3)])
def test_mfma_gram_equals_popcount_gram(monkeypatch, nvars, N, seed):
    cols, dims = _dataset(nvars, N, seed)
    rng = np.random.default_rng(seed + 100)
    x = rng.integers(0, nvars - 1, 1500)
    y = np.minimum(nvars - 1, x + 1 + rng.integers(0, nvars, 1500))
    pairs = np.unique(np.stack([x, y], 1), axis=0)
    pairs = np.concatenate([pairs, [[0, 1], [0, nvars - 1], [nvars - 2, nvars - 1]]]).astype(np.int32)
    got = F.IndependenceTest(F.Dataset(columns=cols, dims=dims)).production_counts(pairs, 0, 16)
    monkeypatch.setenv("FBN_CI_GRAM_NO_MFMA", "1")
    ref = F.IndependenceTest(F.Dataset(columns=cols, dims=dims)).production_counts(pairs, 0, 16)
    np.testing.assert_array_equal(got, ref)
    cells = dims[pairs[:, 0]] * dims[pairs[:, 1]]
    for k in range(0, len(pairs), 97):
        assert got[k, :cells[k]].sum() == N
        # against numpy: the table's multiset of counts (cell order is the kernel's own)
        joint = np.bincount(cols[pairs[k, 0]].astype(np.int64) * dims[pairs[k, 1]] + cols[pairs[k, 1]],
                            minlength=cells[k])
        assert sorted(got[k, :cells[k]].tolist()) == sorted(joint.tolist())
