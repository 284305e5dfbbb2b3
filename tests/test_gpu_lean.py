"""The lean stencil walk (variant bit kVL = 33554432): slices
whose pattern is a subset of one stencil's {-D, -a, -1, 0, +1, +a, +D} and
whose template chunk holds one value per slot are summed from per-class
values (no per-row data), the x-line ends' missing -1 / +1 entries by the
-0.0 identity. Ap must equal the oracle's per-row loop (CG.hpp's
VectorOperations::spmv, VectorOperations.hpp:438-466) bit for bit, with
non-finite and signed-zero x included, in f64 and f32, and CG over it must
match the oracle's iterates.
"""
import ctypes as C

import numpy as np
import pytest

from conjugategradient_amd import CG, Matrix, Vector, VectorOperations
from conjugategradient_amd._native import CgxError, check, lib
from tests.util import rel

pytestmark = pytest.mark.gpu

KVL = 33554432


def lean_info(m):
    c, s, g, d, a, pp = C.c_int(), C.c_int64(), C.c_int(), C.c_int(), C.c_int(), C.c_int()
    check(lib().cgx_csr_lean_info(m.schedule(), C.byref(c), C.byref(s), C.byref(g),
                                  C.byref(d), C.byref(a), C.byref(pp)))
    return c.value, s.value, g.value, d.value, a.value, pp.value


def variant(m):
    v = C.c_int()
    check(lib().cgx_csr_variant(m.schedule(), C.byref(v)))
    return v.value


def spmv(queue, m, x, dtype):
    n = m.N()
    ops = VectorOperations(queue, dtype)
    ops.setVectorSize(n)
    y = Vector(queue, n, dtype=dtype)
    ops.spmv(m, Vector(queue, x, dtype=dtype), y, m.NNZ(), count=n)
    return y.to_numpy()


# (dim, nx, ny, nz), the stencil's (D, a), whether every interior slice is lean
CASES = {
    "p3d_128x64x40": ((3, 128, 64, 40), (8192, 128)),
    "p3d_128x96x40": ((3, 128, 96, 40), (12288, 128)),  # a slice is a whole x-line
    "p3d_256x32x24": ((3, 256, 32, 24), (8192, 256)),
    "p2d_1024x640": ((2, 1024, 640, 1), (1024, 0)),
    # planes of 1,024 slices: the chunked walk where the grid's step is half a plane
    "p3d_512x256x16": ((3, 512, 256, 16), (131072, 512)),
}


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lean_spmv_bitexact(queue, oracle, monkeypatch, case, dtype):
    dims, (D, a) = CASES[case]
    rp, cl, vl = oracle.poisson(*dims)
    n = len(rp) - 1
    # the walk forced at creation (its first grid candidate)
    monkeypatch.setenv("CGX_SPMV_VARIANT", f"{KVL}:0")
    m = Matrix(queue, vl.astype(dtype), cl, rp, dtype=dtype)
    assert variant(m) & KVL
    ncls, nlean, grid, d, aa, chunked = lean_info(m)
    nsl = n // 128
    assert (d, aa) == (D, a)
    assert 1 <= ncls <= 32 and grid % 8 == 0 and grid > 0
    assert nlean >= nsl // 2, (nlean, nsl)  # the interior; boundary lines may run the per-slice form
    x = np.random.default_rng(7).standard_normal(n).astype(dtype)
    nx = dims[1]
    # non-finite and signed-zero values, some at x-line ends (the DPP edges)
    x[[0, nx - 1, nx, 5 * nx + 17, n // 2, n - 1]] = [np.inf, -0.0, np.nan, -np.inf, 0.0, -0.0]
    y = spmv(queue, m, x, dtype)
    if dtype == np.float64:
        want = oracle.spmv(rp, cl, vl, x)
    else:  # the same per-row loop in f32 (products rounded, sums in CSR order)
        want = np.zeros(n, np.float32)
        deg = np.diff(rp)
        v32 = vl.astype(np.float32)
        with np.errstate(invalid="ignore"):
            for j in range(int(deg.max())):
                r = np.nonzero(deg > j)[0]
                k = rp[r] + j
                want[r] = want[r] + v32[k] * x[cl[k]]
    np.testing.assert_array_equal(y, want)


def test_lean_mixed_with_the_per_slice_form(queue, oracle):
    # three rows with a diagonal of their own: their slices' chunks match no
    # template and run the per-slice value-code form inside the lean walk;
    # an x-line length that is no multiple of 128 (slices straddling line
    # ends) has no lean slice at all and is refused
    rp, cl, vl = oracle.poisson(3, 128, 64, 40)
    n = len(rp) - 1
    odd = [1000, 70001, 123456]
    for r in odd:
        k = rp[r] + np.nonzero(cl[rp[r]:rp[r + 1]] == r)[0][0]
        vl[k] = 7.0
    m = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(m.schedule(), 3))
    check(lib().cgx_csr_set_variant(m.schedule(), KVL))
    _, nlean, _, _, _, _ = lean_info(m)
    assert nlean <= n // 128 - len(odd)
    x = np.random.default_rng(3).standard_normal(n)
    np.testing.assert_array_equal(spmv(queue, m, x, np.float64), oracle.spmv(rp, cl, vl, x))
    rp, cl, vl = oracle.poisson(3, 96, 40, 30)
    m = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(m.schedule(), 3))
    with pytest.raises(CgxError, match="lean"):
        check(lib().cgx_csr_set_variant(m.schedule(), KVL))


def test_lean_refused_without_templates(queue, oracle, monkeypatch):
    monkeypatch.setenv("CGX_VT", "0")
    rp, cl, vl = oracle.poisson(3, 32, 32, 32)
    m = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(m.schedule(), 3))
    with pytest.raises(CgxError, match="templates"):
        check(lib().cgx_csr_set_variant(m.schedule(), KVL))


@pytest.mark.parametrize("mode", [1, 3, 4, 6])
def test_lean_in_the_solver(queue, oracle, mode):
    dims = (3, 128, 64, 40)
    rp, cl, vl = oracle.poisson(*dims)
    n = len(rp) - 1
    b = np.arange(1, n + 1, dtype=np.float64)  # Tester.cpp:27-30
    xs = {}
    for v in (KVL, 2050 | 32768 | 262144 | 524288 | 1048576):
        m = Matrix(queue, vl, cl, rp)
        check(lib().cgx_csr_set_sell(m.schedule(), 3))
        check(lib().cgx_csr_set_variant(m.schedule(), v))
        cg = CG(queue)
        cg.mode = 3 if mode == 6 and v != KVL else mode  # (mode 6: the lean walk only)
        cg.setMatrix(m)
        cg.setTarget(b)
        cg.solve(0.0, max_iter=45)
        assert cg.iterations == 45
        xs[v] = cg.extract()
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 45, 8)
    assert rel(xs[KVL], xr) <= 1e-10
    # the SpMV is the same; p.Ap's partials split differently, but the dots
    # are double-length sums (round 6): bit for bit
    np.testing.assert_array_equal(xs[KVL], xs[2050 | 32768 | 262144 | 524288 | 1048576])


def test_lean_modes_3_and_1_bit_identical(queue, oracle):
    """Modes 3 and 4 (x deferred over four bodies; mode 4 forms p_k inside
    k_spmv_fd_lean, on the walk's own grid) against mode 1, solved to
    tolerances whose body counts end in every slot of a 4-body group: body
    count, x and final r.r bit for bit, and the oracle's body count."""
    rp, cl, vl = oracle.poisson(3, 128, 64, 40)
    n = len(rp) - 1
    b = np.arange(1, n + 1, dtype=np.float64)
    m = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(m.schedule(), 3))
    check(lib().cgx_csr_set_variant(m.schedule(), KVL))
    slots = set()
    for tol in (1e-4, 3e-6, 1e-7, 1e-8, 3e-9, 1e-10):
        out = {}
        for mode in (1, 3, 4, 6):
            cg = CG(queue)
            cg.mode = mode
            cg.setMatrix(m)
            cg.setTarget(b)
            cg.solve(tol * float(np.linalg.norm(b)))
            out[mode] = (cg.iterations, cg.extract(), cg.final_rxr)
        for mode in (3, 4, 6):
            assert out[mode][0] == out[1][0], (tol, mode)
            np.testing.assert_array_equal(out[mode][1], out[1][1])
            assert out[mode][2] == out[1][2]
        slots.add(out[1][0] % 4)
        if tol == 1e-8:
            _, res = oracle.cg_solve_omp(rp, cl, vl, b, tol * float(np.linalg.norm(b)), 8)
            assert abs(out[1][0] - res.iterations) <= 2
    assert len(slots) >= 3, slots


def set_team(m, on=1):
    check(lib().cgx_csr_set_lean_team(m.schedule(), on))
    t = C.c_int()
    check(lib().cgx_csr_lean_team(m.schedule(), C.byref(t)))
    assert t.value == on


@pytest.mark.parametrize("dims", [(3, 128, 64, 40), (3, 512, 256, 16)], ids=["plane", "chunked"])
def test_lean_team_in_the_solver(queue, oracle, monkeypatch, dims):
    """Mode 4's fused walk in its team form (k_spmv_fd_lean_t: 16 waves per
    workgroup, the published pairs are the formed p_k): 45 bodies against
    the oracle's iterates and against mode 1 (its p.Ap partials split over a
    quarter of the workgroups: one dot summed in another order, so to
    rounding), the 4-wave form bit for bit where it is the same launch shape
    (mode 4 without the team form equals mode 1), and a tolerance stop at
    the oracle's body count."""
    rp, cl, vl = oracle.poisson(*dims)
    n = len(rp) - 1
    b = np.arange(1, n + 1, dtype=np.float64)  # Tester.cpp:27-30
    monkeypatch.setenv("CGX_SPMV_VARIANT", f"{KVL}:0")
    m = Matrix(queue, vl, cl, rp)
    xs = {}
    for mode, team in ((1, 0), (4, 0), (4, 1)):
        set_team(m, team)
        cg = CG(queue)
        cg.mode = mode
        cg.setMatrix(m)
        cg.setTarget(b)
        cg.solve(0.0, max_iter=45)
        assert cg.iterations == 45
        xs[(mode, team)] = cg.extract()
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 45, 8)
    np.testing.assert_array_equal(xs[(4, 0)], xs[(1, 0)])
    assert rel(xs[(4, 1)], xr) <= 1e-10, rel(xs[(4, 1)], xr)
    np.testing.assert_array_equal(xs[(4, 1)], xs[(1, 0)])  # double-length dots (round 6)
    tol = 1e-8 * float(np.linalg.norm(b))
    set_team(m, 1)
    cg = CG(queue)
    cg.mode = 4
    cg.setMatrix(m)
    cg.setTarget(b)
    cg.solve(tol)
    x4 = cg.extract()
    xo, res = oracle.cg_solve_omp(rp, cl, vl, b, tol, 8)
    assert abs(cg.iterations - res.iterations) <= 2
    assert rel(x4, xo) <= 1e-10
