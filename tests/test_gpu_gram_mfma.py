"""The level-0 Gram on the gfx950 matrix cores (ci_gram_mfma.hip: FP4 one-hot x FP4 MFMA, split-K
uint16 slabs) on ragged shapes -- leading-row counts that are not multiples of the 256-row tile,
sample counts that are not multiples of the 128-sample stage, mixed state counts:

* against the UNMODIFIED reference's Counts2D::FillTable (src/CellTable.cpp:430-455) on a seeded
  sample of the pairs, tile-edge pairs included (tests/golden/gram_ragged.ci.gz, oracle/_ref/ref_dump
  ci, tests/golden/make_golden_synth.py gram), for the MFMA Gram (default) and the popcount Gram
  (FBN_CI_GRAM_NO_MFMA) alike;
* against the popcount Gram on every pair of the test (every level-0 pair table identical, each
  summing to N).

Config 5 itself is pinned against the reference's tables in test_gpu_pc_c5_pinned.py."""
import os

import numpy as np
import pytest
from conftest import GOLD, GRAM_SHAPES, fnv1a_columns, gram_dataset, read_ci_blocks

import fastbn_amd as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ref_blocks():
    return read_ci_blocks(os.path.join(GOLD, "gram_ragged.ci.gz"))


@pytest.mark.parametrize("nvars,N,seed", GRAM_SHAPES)
@pytest.mark.parametrize("gram", ["mfma", "popcount"])
def test_gram_pair_tables_equal_reference_counts2d(monkeypatch, ref_blocks, nvars, N, seed, gram):
    cols, dims, _ = gram_dataset(nvars, N, seed)
    rdims, colhash, tests = ref_blocks[(nvars, N, seed)]
    assert rdims == dims.tolist()
    h = fnv1a_columns(cols)
    assert all(int(h[v]) == colhash[v] for v in range(nvars))  # the reference read these columns
    if gram == "popcount":
        monkeypatch.setenv("FBN_CI_GRAM_NO_MFMA", "1")
    items = np.array([[x, y] for x, y, _, _ in tests], np.int32)
    got = F.IndependenceTest(F.Dataset(columns=cols, dims=dims)).production_counts(items, 0, 16)
    for k, (x, y, _, ref) in enumerate(tests):
        np.testing.assert_array_equal(got[k, :len(ref)], ref, err_msg=f"pair ({x}, {y}) of shape {nvars}x{N}")


@pytest.mark.parametrize("nvars,N,seed", GRAM_SHAPES)
def test_mfma_gram_equals_popcount_gram(monkeypatch, nvars, N, seed):
    cols, dims, pairs = gram_dataset(nvars, N, seed)
    got = F.IndependenceTest(F.Dataset(columns=cols, dims=dims)).production_counts(pairs, 0, 16)
    monkeypatch.setenv("FBN_CI_GRAM_NO_MFMA", "1")
    ref = F.IndependenceTest(F.Dataset(columns=cols, dims=dims)).production_counts(pairs, 0, 16)
    np.testing.assert_array_equal(got, ref)
    cells = dims[pairs[:, 0]] * dims[pairs[:, 1]]
    for k in range(0, len(pairs), 97):
        assert got[k, :cells[k]].sum() == N
