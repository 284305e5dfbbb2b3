"""SELL-64 SpMV format (variant bit 2048) against the oracle.

cgx_csr_create builds a SELL-64 copy of a matrix whose 64-row slices have at
most 64 distinct (col - row) offsets (stencils, banded matrices). Rows are
summed in CSR order in a register, so the bar is the same as the CSR-stream
kernels': bit-exact with the oracle's restatement of the reference SpMV.
Matrices that do not qualify keep only the CSR-stream schedule and refuse a
SELL variant.
"""
import ctypes as C

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd import Matrix, Vector, VectorOperations
from conjugategradient_amd._native import CgxError, check, lib
from tests.util import coo_to_csr, irregular_spd, rel

pytestmark = pytest.mark.gpu

VARIANTS = [2048, 2050, 2056, 2058, 6144, 6146, 8192, 8194, 13, 15, 0]


def banded(n, half=6, seed=1, empty_every=0):
    """Random symmetric banded SPD matrix (offsets within +-half): qualifies
    for SELL with ragged rows; optional empty rows."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for d in range(1, half + 1):
        keep = rng.random(n - d) < 0.92
        i = np.nonzero(keep)[0]
        rows += [i, i + d]
        cols += [i + d, i]
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    vals = -rng.uniform(0.5, 1.5, len(rows))
    if empty_every:
        dead = (rows % empty_every == 0) | (cols % empty_every == 0)
        rows, cols, vals = rows[~dead], cols[~dead], vals[~dead]
    deg = np.zeros(n)
    np.add.at(deg, rows, -vals)
    diag = np.arange(n)
    live = deg > 0 if empty_every else np.ones(n, bool)
    rows = np.concatenate([rows, diag[live]])
    cols = np.concatenate([cols, diag[live]])
    vals = np.concatenate([vals, deg[live] + 0.1])
    return coo_to_csr(n, rows, cols, vals)


def _matrix_cases(oracle):
    return {
        "poisson2d": oracle.poisson(2, 96, 80, 1),
        "poisson3d_ragged": oracle.poisson(3, 23, 19, 17),     # n % 64 != 0
        # planes of 33,280 rows (> 256 slices): the host builds a visit order
        "poisson3d_wide": oracle.poisson(3, 256, 130, 3),
        "banded": banded(10_007, half=9),
        "empty_rows": banded(3_001, half=6, empty_every=13),
        "tiny": (np.array([0, 1, 3, 4], np.int32), np.array([0, 0, 1, 2], np.int32),
                 np.array([2.0, -1.0, 3.0, 4.0])),
    }


def _sell_info(m):
    has = C.c_int()
    padded = C.c_int64()
    check(lib().cgx_csr_sell_info(m.schedule(), C.byref(has), C.byref(padded)))
    return has.value, padded.value


@pytest.mark.parametrize("R", [1, 2, 3])   # 3: SELL-P
@pytest.mark.parametrize("case", ["poisson2d", "poisson3d_ragged", "poisson3d_wide", "banded",
                                  "empty_rows", "tiny"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sell_spmv_bitexact_all_variants(queue, oracle, case, dtype, R):
    rp, cl, vl = _matrix_cases(oracle)[case]
    n = len(rp) - 1
    A = Matrix(queue, vl, cl, rp, dtype=dtype)
    check(lib().cgx_csr_set_sell(A.schedule(), R))
    has, padded = _sell_info(A)
    assert has == R, case
    assert len(vl) <= padded <= len(vl) + len(vl) // 4 + 4096 + 64 * np.diff(rp).max()
    x = np.random.default_rng(3).standard_normal(n)
    if dtype == np.float32:
        want = (vl.astype(np.float32), x.astype(np.float32))
    ops = VectorOperations(queue, dtype)
    ops.setVectorSize(n)
    xv = Vector(queue, x, dtype=dtype)
    ref = oracle.spmv(rp, cl, vl, x) if dtype == np.float64 else None
    outs = {}
    for v in VARIANTS:
        check(lib().cgx_csr_set_variant(A.schedule(), v))
        yv = Vector(queue, n, dtype=dtype)
        ops.spmv(A, xv, yv, A.NNZ(), count=n)
        outs[v] = yv.to_numpy()
    for v in VARIANTS:
        if ref is not None:
            np.testing.assert_array_equal(outs[v], ref, err_msg=f"variant {v}")
        else:   # f32: every variant computes the same per-row f32 sum
            np.testing.assert_array_equal(outs[v], outs[0], err_msg=f"variant {v}")
    if dtype == np.float32:
        # and that f32 sum is the ascending-order f32 row sum
        vf, xf = want
        y = np.zeros(n, np.float32)
        for i in range(0, n, max(1, n // 97)):
            s = np.float32(0)
            for k in range(rp[i], rp[i + 1]):
                s = np.float32(s + np.float32(vf[k] * xf[cl[k]]))
            y[i] = s
            assert outs[2048][i] == s


def test_sell_not_built_for_scattered_matrix(queue):
    rp, cl, vl = irregular_spd(20_000, seed=4)
    A = Matrix(queue, vl, cl, rp)
    has, _ = _sell_info(A)
    assert has == 0
    check(lib().cgx_csr_set_sell(A.schedule(), 2))
    assert _sell_info(A)[0] == 0
    with pytest.raises(CgxError, match="SELL"):
        check(lib().cgx_csr_set_variant(A.schedule(), 2048))
    with pytest.raises(CgxError, match="unknown"):
        check(lib().cgx_csr_set_variant(A.schedule(), 9999))


def test_sell_dropped_on_request(queue, oracle):
    rp, cl, vl = oracle.poisson(2, 32, 32, 1)
    A = Matrix(queue, vl, cl, rp)
    assert _sell_info(A)[0] == 3
    check(lib().cgx_csr_set_sell(A.schedule(), 0))
    assert _sell_info(A)[0] == 0
    v = C.c_int()
    check(lib().cgx_csr_variant(A.schedule(), C.byref(v)))
    assert not v.value & (2048 | 8192)


@pytest.mark.parametrize("R", [1, 2, 3])
def test_sell_spmv_nonfinite_and_signed_zero(queue, oracle, R):
    # padding entries are dropped, not multiplied: an Inf/NaN in x reaches
    # exactly the rows whose real entries touch it, and -0 sums stay -0
    rp, cl, vl = oracle.poisson(2, 16, 12, 1)
    n = len(rp) - 1
    x = np.zeros(n)
    x[5] = np.inf
    x[77] = np.nan
    x[100] = -0.0
    A = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(A.schedule(), R))
    check(lib().cgx_csr_set_variant(A.schedule(), 2048))
    ops = VectorOperations(queue)
    ops.setVectorSize(n)
    yv = Vector(queue, n)
    ops.spmv(A, Vector(queue, x), yv, A.NNZ(), count=n)
    y = yv.to_numpy()
    ref = oracle.spmv(rp, cl, vl, x)
    np.testing.assert_array_equal(np.isnan(y), np.isnan(ref))
    np.testing.assert_array_equal(y[~np.isnan(ref)], ref[~np.isnan(ref)])
    np.testing.assert_array_equal(np.signbit(y), np.signbit(ref))


@pytest.mark.parametrize("sell", ["1", "2", "3", "0"])
@pytest.mark.parametrize("dim,n", [(2, 64), (3, 20), (3, 0)])
def test_cg_both_formats_match_oracle(oracle, sell, dim, n):
    # n = 0: 256 x 130 x 3, wide planes
    rp, cl, vl = oracle.poisson(dim, n, n, n) if n else oracle.poisson(3, 256, 130, 3)
    b = np.arange(1, len(rp), dtype=np.float64)
    cg = cga.CG.createCG()
    cg.setMatrix(vl, cl, rp)
    check(lib().cgx_csr_set_sell(cg.A.schedule(), int(sell)))
    cg.setTarget(b)
    cg.solve(1e-8)
    v = C.c_int()
    check(lib().cgx_csr_variant(cg.A.schedule(), C.byref(v)))
    assert bool(v.value & (2048 | 8192)) == (sell != "0")
    assert _sell_info(cg.A)[0] == int(sell)
    xr, res = oracle.cg_solve(rp, cl, vl, b, 1e-8)
    assert abs(cg.iterations - res.iterations) <= 2
    assert rel(cg.extract(), xr) <= 1e-10


def test_auto_visit_order_on_large_planes(queue, oracle, monkeypatch):
    """Planes of >= 1,024 slices get the chunked visit order without any
    request (cgx_abi.cpp build_sell; 512^3: SpMV 793 -> 710 us): the SpMV
    stays bit-exact against the oracle in the production form and in
    CSR-stream, and CG holds the oracle's iterates (only the p.Ap partials'
    grouping changes)."""
    rp, cl, vl = oracle.poisson(3, 512, 256, 4)  # planes of 131,072 rows = 1,024 slices
    n = len(rp) - 1
    A = Matrix(queue, vl, cl, rp)
    v = C.c_int()
    check(lib().cgx_csr_variant(A.schedule(), C.byref(v)))
    prod = v.value
    assert prod & 8192, prod  # SELL-P (the ordered walk)
    o = C.c_int(-1)
    check(lib().cgx_csr_visit_order(A.schedule(), C.byref(o)))
    assert o.value == 1
    x = np.random.default_rng(11).standard_normal(n)
    ref = oracle.spmv(rp, cl, vl, x)
    ops = VectorOperations(queue)
    ops.setVectorSize(n)
    xv = Vector(queue, x)
    for var in (prod, 15):
        check(lib().cgx_csr_set_variant(A.schedule(), var))
        yv = Vector(queue, n)
        ops.spmv(A, xv, yv, A.NNZ(), count=n)
        np.testing.assert_array_equal(yv.to_numpy(), ref, err_msg=f"variant {var}")
    check(lib().cgx_csr_set_variant(A.schedule(), prod))
    b = np.arange(1, n + 1, dtype=np.float64)
    cg = cga.CG(queue)
    cg.setMatrix(A)
    cg.setTarget(b)
    cg.solve(0.0, max_iter=30)
    xr, res = oracle.cg_solve(rp, cl, vl, b, 0.0, max_iter=30)
    assert cg.iterations == res.iterations
    assert rel(cg.extract(), xr) <= 1e-12
