"""Plane-march SpMV (variant bit 2097152) against the oracle.

The march form walks the slices of one column through a run of planes and
takes the x pairs at -D and +D from the previous and next slice's center
pair in registers (cgx_kernels.hip spmv_sellpv_march). Its row sums run in
the same slot order as every SELL-P form, so the bar is bit-exactness with
the oracle's restatement of the reference SpMV (VectorOperations.hpp:438-466)
on every geometry the plan accepts (3-D 7-point and 2-D 5-point with the
plane a multiple of 128 rows, ragged last planes) and a silent fallback to
the per-slice form where it does not apply.
"""
import ctypes as C

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd import Matrix
from conjugategradient_amd._native import check, lib
from tests.test_gpu_value_codes import spmv_all
from tests.util import rel

pytestmark = pytest.mark.gpu

# march on the pipelined stencil form: 8-bit codes (default / nt loads),
# 4-bit codes (default / nt loads)
MARCH = [3710976, 3710978, 3973120, 3973122]
STENCIL = [1613826, 1875970]  # the same forms without the march
PLAIN = 8194


def march_info(A):
    k, a, ln = C.c_int(), C.c_int(), C.c_int()
    check(lib().cgx_csr_march_info(A.schedule(), C.byref(k), C.byref(a), C.byref(ln)))
    return k.value, a.value, ln.value


# (dim, nx, ny, nz, expected stride K = nx*ny/128 (3-D) or nx/128 (2-D), a)
GEOMS = [
    (3, 32, 32, 20, 8, 32),     # K = 8
    (3, 16, 8, 30, 1, 16),      # K = 1: a column is every slice of the run
    (3, 64, 64, 40, 32, 64),
    (3, 32, 16, 13, 4, 32),     # odd plane count
    (3, 128, 7, 12, 7, 128),    # a = nx = one slice: the +-a gathers are whole slices
    (2, 256, 100, 1, 2, 0),
    (2, 128, 77, 1, 1, 0),
    (2, 384, 50, 1, 3, 0),
]


@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: "x".join(map(str, g[:4])))
def test_march_spmv_bitexact(queue, oracle, geom):
    dim, nx, ny, nz, K, a = geom
    rp, cl, vl = oracle.poisson(dim, nx, ny, nz)
    n = len(rp) - 1
    A = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    assert march_info(A) == (K, a, 0)  # run length 0: fill the grid's waves
    x = np.random.default_rng(11).standard_normal(n)
    out = spmv_all(queue, A, x, MARCH + STENCIL + [PLAIN])
    ref = oracle.spmv(rp, cl, vl, x)
    for v in MARCH + STENCIL + [PLAIN]:
        np.testing.assert_array_equal(out[v], ref, err_msg=f"variant {v}")


def test_march_spmv_float32(queue, oracle):
    rp, cl, vl = oracle.poisson(3, 32, 32, 11)
    n = len(rp) - 1
    A = Matrix(queue, vl, cl, rp, dtype=np.float32)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    assert march_info(A)[0] == 8
    x = np.random.default_rng(2).standard_normal(n)
    out = spmv_all(queue, A, x, MARCH + [PLAIN], np.float32)
    for v in MARCH:
        np.testing.assert_array_equal(out[v], out[PLAIN], err_msg=f"variant {v}")


@pytest.mark.parametrize("dims", [(3, 23, 19, 17), (3, 20, 20, 20), (2, 100, 90, 1)])
def test_march_not_planned(queue, oracle, dims):
    """A plane that is not a multiple of 128 rows has no march plan; the
    march variant then runs the per-slice stencil form, still bit-exact."""
    rp, cl, vl = oracle.poisson(*dims)
    A = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    assert march_info(A) == (0, 0, 0)
    x = np.random.default_rng(4).standard_normal(len(rp) - 1)
    out = spmv_all(queue, A, x, MARCH[-1:])
    np.testing.assert_array_equal(out[MARCH[-1]], oracle.spmv(rp, cl, vl, x))


def test_march_nonfinite_x(queue, oracle):
    """Inf / NaN / -0.0 in x: an empty slot is skipped, never multiplied."""
    rp, cl, vl = oracle.poisson(3, 16, 16, 12)
    n = len(rp) - 1
    x = np.random.default_rng(9).standard_normal(n)
    x[[5, 300, 1500, 2047]] = [np.inf, np.nan, -0.0, -np.inf]
    A = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    y = spmv_all(queue, A, x, MARCH)
    ref = oracle.spmv(rp, cl, vl, x)
    for v in MARCH:
        np.testing.assert_array_equal(np.isnan(y[v]), np.isnan(ref))
        ok = ~np.isnan(ref)
        np.testing.assert_array_equal(y[v][ok], ref[ok])


@pytest.mark.parametrize("dims", [(3, 32, 32, 24), (2, 256, 90, 1)])
def test_cg_march_in_the_loop(oracle, monkeypatch, dims):
    """The march form forced into the CG loop (k_cg_init, k_spmv_dot) against
    the oracle (SURVEY §8(c) tolerances: ±2 bodies at 1e-8, 1e-10 relative).
    Its p.Ap partials group rows per wave differently from the consecutive
    walk, so x is held to the tolerance, not to the other forms' bits."""
    dim, nx, ny, nz = dims
    rp, cl, vl = oracle.poisson(dim, nx, ny, nz)
    b = np.arange(1, len(rp), dtype=np.float64)
    monkeypatch.setenv("CGX_SPMV_VARIANT", str(MARCH[-1]))
    cg = cga.CG.createCG()
    cg.setMatrix(vl, cl, rp)
    cg.setTarget(b)
    v = C.c_int()
    check(lib().cgx_csr_variant(cg.A.schedule(), C.byref(v)))
    assert v.value & 2097152, v.value
    cg.solve(1e-8)
    xr, res = oracle.cg_solve(rp, cl, vl, b, 1e-8)
    assert abs(cg.iterations - res.iterations) <= 2
    assert rel(cg.extract(), xr) <= 1e-10
