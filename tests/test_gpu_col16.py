"""CSR-stream on 16-bit column deltas (variant bit 128: 133 / 135 are the
paired loop 5 / 7 reading each entry's column as its offset from the row
block's first row, 10 bytes per entry instead of 12). The row sums are the
reference's per-row loop (VectorOperations.hpp:456-459) in either form, so
Ap is bit-identical to the int32 form and to the oracle; a matrix with a
column more than 32767 rows from its block's first row refuses the form."""
import ctypes as C

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd._native import check, lib
from tests.util import coo_to_csr, irregular_spd, rel

pytestmark = pytest.mark.gpu


def _spmv(queue, m, x):
    y = cga.Vector(queue, m.N())
    cga.VectorOperations(queue).spmv(m, cga.Vector(queue, x), y, m.NNZ(), count=m.N())
    return y.to_numpy()


@pytest.mark.parametrize("v", [133, 135])
@pytest.mark.parametrize("case", ["irr", "irr_hub", "odd_blocks"])
def test_col16_spmv_bitexact(queue, oracle, case, v):
    if case == "irr":
        rp, cl, vl = irregular_spd(120_000, seed=7)
    elif case == "irr_hub":  # a row longer than a tile: its own block, int32 columns
        rp, cl, vl = irregular_spd(50_000, seed=8, hub=5000)
    else:  # rows of 1..9 entries: blocks start at odd entries (the pair before k0)
        rng = np.random.default_rng(9)
        n = 40_000
        deg = rng.integers(0, 9, n)
        rows = np.repeat(np.arange(n), deg)
        cols = np.clip(rows + rng.integers(-3000, 3000, len(rows)), 0, n - 1)
        rows = np.concatenate([rows, np.arange(n)])
        cols = np.concatenate([cols, np.arange(n)])
        vals = rng.standard_normal(len(rows))
        rp, cl, vl = coo_to_csr(n, rows, cols, vals)
    m = cga.Matrix(queue, vl, cl, rp)
    x = np.random.default_rng(1).standard_normal(len(rp) - 1)
    want = oracle.spmv(rp, cl, vl, x)
    check(lib().cgx_csr_set_variant(m.schedule(), v))
    got = C.c_int()
    check(lib().cgx_csr_variant(m.schedule(), C.byref(got)))
    assert got.value == v
    y = _spmv(queue, m, x)
    # a row longer than a tile is tree-summed by a workgroup of its own in
    # every CSR-stream form (1e-12, test_gpu_kernels.py); the rest bit-exact
    long = np.diff(rp) > 2042
    np.testing.assert_array_equal(y[~long], want[~long])
    assert np.allclose(y[long], want[long], rtol=1e-12, atol=0)
    sb = C.c_int64()
    check(lib().cgx_csr_stream_bytes(m.schedule(), C.byref(sb)))
    assert sb.value == 10 * m.NNZ() + 4 * (m.N() + 1)


def test_col16_refused_for_far_columns(queue):
    n = 100_000  # row 0 couples to row n - 1: a delta of 99,999
    rows = np.concatenate([np.arange(n), [0, n - 1]])
    cols = np.concatenate([np.arange(n), [n - 1, 0]])
    vals = np.concatenate([np.full(n, 4.0), [-1.0, -1.0]])
    rp, cl, vl = coo_to_csr(n, rows, cols, vals)
    m = cga.Matrix(queue, vl, cl, rp)
    assert lib().cgx_csr_set_variant(m.schedule(), 133) != 0
    assert b"16-bit column deltas" in lib().cgx_last_error()


def test_col16_cg_matches_oracle(queue, oracle, monkeypatch):
    monkeypatch.setenv("CGX_SPMV_VARIANT", "133")
    rp, cl, vl = irregular_spd(60_000, seed=11, shift=10.0)
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, len(rp), dtype=np.float64)
    cg = cga.CG(queue)
    cg.mode = 3
    cg.setMatrix(m)
    cg.setTarget(b)
    cg.solve(0.0, max_iter=40)
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 40, 8)
    assert cg.iterations == 40 and rel(cg.extract(), xr) <= 1e-10
