"""Parity of the gfx950 kernels (through libcgx's C ABI) with the oracle.

Bars: SpMV / AXPY / generator are bit-exact (same per-row and
per-element arithmetic, no FMA); dots are reductions in a different order,
so they are compared at 1e-13 relative; CG solutions at
||dx||/||x|| <= 1e-10 with iteration counts within +-2 at tol 1e-8.
"""
import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd import Matrix, Scalar, Vector, VectorOperations
from tests.util import irregular_spd, rel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dim,nx,ny,nz", [(2, 16, 16, 1), (2, 33, 17, 1), (3, 16, 16, 16),
                                          (3, 7, 5, 3), (3, 1, 1, 5), (2, 1, 9, 1)])
def test_poisson_generator_matches_oracle(queue, oracle, dim, nx, ny, nz):
    rp, cl, vl = oracle.poisson(dim, nx, ny, nz)
    m = Matrix.poisson(queue, dim, nx, ny, nz)
    assert m.N() == len(rp) - 1 and m.NNZ() == len(vl)
    np.testing.assert_array_equal(m.rows().download(), rp)
    np.testing.assert_array_equal(m.columns().download(), cl)
    np.testing.assert_array_equal(m.data().download(), vl)


def _spmv(queue, rp, cl, vl, x, dtype=np.float64):
    A = Matrix(queue, vl, cl, rp, dtype=dtype)
    xv = Vector(queue, x, dtype=dtype)
    yv = Vector(queue, len(rp) - 1, dtype=dtype)
    ops = VectorOperations(queue, dtype)
    ops.setVectorSize(len(rp) - 1)
    ops.spmv(A, xv, yv, A.NNZ(), count=len(rp) - 1)
    return yv.to_numpy()


@pytest.mark.parametrize("case", ["poisson2d", "poisson3d", "irregular", "single_row"])
def test_spmv_bitexact(queue, oracle, case):
    rng = np.random.default_rng(7)
    if case == "poisson2d":
        rp, cl, vl = oracle.poisson(2, 128, 128, 1)
    elif case == "poisson3d":
        rp, cl, vl = oracle.poisson(3, 24, 20, 18)
    elif case == "irregular":
        rp, cl, vl = irregular_spd(50_000, seed=3)
    else:
        rp, cl, vl = np.array([0, 3], np.int32), np.array([0, 0, 0], np.int32), np.ones(3)
    x = rng.standard_normal(len(rp) - 1)
    y = _spmv(queue, rp, cl, vl, x)
    np.testing.assert_array_equal(y, oracle.spmv(rp, cl, vl, x))


def test_spmv_long_row(queue, oracle):
    # one row with 5000 entries (> one 2048-entry tile) takes the tree path:
    # its sum is reassociated, every other row stays bit-exact
    rp, cl, vl = irregular_spd(20_000, seed=5, hub=5000)
    lens = np.diff(rp)
    assert lens.max() > 2048
    x = np.random.default_rng(1).standard_normal(len(rp) - 1)
    y = _spmv(queue, rp, cl, vl, x)
    yr = oracle.spmv(rp, cl, vl, x)
    long = lens > 2048
    np.testing.assert_array_equal(y[~long], yr[~long])
    np.testing.assert_allclose(y[long], yr[long], rtol=1e-12, atol=1e-12)


def test_spmv_f32(queue, oracle):
    rp, cl, vl = oracle.poisson(2, 64, 64, 1)
    x = np.random.default_rng(2).standard_normal(len(rp) - 1).astype(np.float32)
    y = _spmv(queue, rp, cl, vl, x, dtype=np.float32)
    yr = oracle.spmv(rp, cl, vl, x.astype(np.float64))
    np.testing.assert_allclose(y, yr, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n", [1, 2, 255, 256, 4097, 1_000_003])
def test_dot_and_norm_accumulate(queue, oracle, n):
    rng = np.random.default_rng(n)
    x, y = rng.standard_normal(n), rng.standard_normal(n)
    ops = VectorOperations(queue)
    ops.setVectorSize(n)
    xv, yv = Vector(queue, x), Vector(queue, y)
    s = Scalar(queue, 5.0)                     # accumulate semantics (Q4)
    ops.dot_product_trivial(xv, yv, s)
    want = oracle.dot_acc(x, y, 5.0)
    assert abs(s.get() - want) <= 1e-13 * (abs(want) + np.abs(x * y).sum())
    s2 = Scalar(queue, 0.0)
    ops.norm(xv, s2)
    assert s2.get() == pytest.approx(oracle.norm_acc(x, 0.0), rel=1e-13)


@pytest.mark.parametrize("n", [1, 3, 1024, 100_001])
def test_axpy_bitexact(queue, oracle, n):
    rng = np.random.default_rng(11)
    x, y = rng.standard_normal(n), rng.standard_normal(n)
    a, b = 0.7310585786300049, -1.3862943611198906
    ops = VectorOperations(queue)
    ops.setVectorSize(n)
    xv, yv, rv = Vector(queue, x), Vector(queue, y), Vector(queue, n)
    sa, sb = Scalar(queue, a), Scalar(queue, b)
    ops.sapbx(xv, yv, sb, rv)
    np.testing.assert_array_equal(rv.to_numpy(), oracle.sapbx(x, y, b))
    ops.sambx(xv, yv, sb, rv)
    np.testing.assert_array_equal(rv.to_numpy(), oracle.sambx(x, y, b))
    ops.saxpby(xv, yv, sa, sb, rv)
    np.testing.assert_array_equal(rv.to_numpy(), oracle.saxpby(x, y, a, b))
    ops.sapbx(xv, yv, sb, xv)                  # in-place alias (CG.hpp:390)
    np.testing.assert_array_equal(xv.to_numpy(), oracle.sapbx(x, y, b))


def _solve(rp, cl, vl, b, tol, **kw):
    cg = cga.CG.createCG()
    cg.setMatrix(vl, cl, rp)
    cg.setTarget(b)
    cg.solve(tol, **kw)
    return cg


@pytest.mark.parametrize("dim,n", [(2, 16), (2, 128), (3, 16)])
def test_cg_solve_matches_oracle(oracle, dim, n):
    rp, cl, vl = oracle.poisson(dim, n, n, n)
    b = np.arange(1, len(rp), dtype=np.float64)       # Tester.cpp:29-30
    for tol in (1e-8, 1e-24):
        cg = _solve(rp, cl, vl, b, tol)
        x = cg.extract()
        xr, res = oracle.cg_solve(rp, cl, vl, b, tol)
        assert rel(x, xr) <= 1e-10, (tol, cg.iterations, res.iterations)
        if tol == 1e-8:
            assert abs(cg.iterations - res.iterations) <= 2
        acc = cg.accuracy()
        assert acc == pytest.approx(oracle.accuracy(rp, cl, vl, b, x), rel=1e-6, abs=1e-30)
        assert acc < 1e-20


def test_cg_irregular(oracle):
    # ill-conditioned (shift 1e-2): the iteration count reacts to the dot
    # products' summation order, so the bar is solution quality, not +-2
    rp, cl, vl = irregular_spd(30_000, seed=9)
    b = np.arange(1, len(rp), dtype=np.float64)
    cg = _solve(rp, cl, vl, b, 1e-6)
    xr, res = oracle.cg_solve(rp, cl, vl, b, 1e-6)
    x = cg.extract()
    print("irregular iterations gpu", cg.iterations, "oracle", res.iterations,
          "rel", rel(x, xr))
    assert abs(cg.iterations - res.iterations) <= max(2, res.iterations // 20)
    assert rel(x, xr) <= 1e-6
    r = oracle.spmv(rp, cl, vl, x) - b
    assert np.linalg.norm(r) <= 10 * max(np.linalg.norm(oracle.spmv(rp, cl, vl, xr) - b), 1e-6)


def test_cg_cap_and_initial_guess(oracle):
    rp, cl, vl = oracle.poisson(2, 40, 40, 1)
    b = np.arange(1, len(rp), dtype=np.float64)
    cg = _solve(rp, cl, vl, b, 1e-30, max_iter=7)
    assert cg.iterations == 7
    xr, res = oracle.cg_solve(rp, cl, vl, b, 1e-30, max_iter=7)
    assert res.iterations == 7 and rel(cg.extract(), xr) <= 1e-12
    # warm start continues from x (CG.hpp:215-219)
    x0 = cg.extract()
    cg2 = cga.CG.createCG()
    cg2.setMatrix(vl, cl, rp)
    cg2.setTarget(b)
    cg2.setInital(x0)
    cg2.solve(1e-8)
    xr2, res2 = oracle.cg_solve(rp, cl, vl, b, 1e-8, x0=x0)
    assert abs(cg2.iterations - res2.iterations) <= 2
    assert rel(cg2.extract(), xr2) <= 1e-10


def test_cg_tol_zero_runs_to_cap_or_nan(oracle):
    # Q5: with improvement 0 the loop runs until r.r underflows; then alpha is
    # 0/0 and x turns NaN, or the N+1 cap ends it (CG.hpp:401,436).
    rp, cl, vl = oracle.poisson(2, 8, 8, 1)
    b = np.arange(1, len(rp), dtype=np.float64)
    cg = _solve(rp, cl, vl, b, 0.0)
    xr, res = oracle.cg_solve(rp, cl, vl, b, 0.0)
    assert cg.iterations <= len(rp)          # at most N + 1 bodies
    assert np.isnan(cg.extract()).any() == np.isnan(xr).any()


def test_cg_f32(oracle):
    rp, cl, vl = oracle.poisson(2, 32, 32, 1)
    b = np.arange(1, len(rp), dtype=np.float64)
    cg = cga.CG.createCG(dtype=np.float32)
    cg.setMatrix(vl, cl, rp)
    cg.setTarget(b)
    cg.solve(1e-2, max_iter=200)
    xr, _ = oracle.cg_solve(rp, cl, vl, b, 1e-12)
    assert rel(cg.extract().astype(np.float64), xr) < 1e-3


def test_errors(queue):
    cg = cga.CG.createCG()
    with pytest.raises(RuntimeError, match="No right hand side"):
        cg.solve(1e-8)
    cg.setTarget(np.ones(4))
    with pytest.raises(RuntimeError, match="No Matrix"):
        cg.solve(1e-8)


def _run_modes(rp, cl, vl, b, tol, max_iter=-1, poll=32, graph=True, modes=(1, 2, 3, 4)):
    out = {}
    for mode in modes:
        cg = cga.CG.createCG()
        cg.mode = mode
        cg.poll_every = poll
        cg.use_graph = graph
        cg.setMatrix(vl, cl, rp)
        cg.setTarget(b)
        cg.solve(tol, max_iter=max_iter)
        out[mode] = (cg.extract(), cg.iterations, cg.final_rxr)
    return out


@pytest.mark.parametrize("case,tol,poll,graph", [("p2d", 1e-8, 32, True), ("p3d", 1e-24, 8, False),
                                                  ("irr", 1e-6, 4, True), ("p2d", 0.0, 32, True)])
def test_fused_iteration_bit_identical_to_three_kernels(oracle, case, tol, poll, graph):
    """Mode 3 defers the x update to every fourth body; every value it
    computes is the same expression, in the same order, as mode 1's, so x is
    bit-identical. Mode 2 (fused) keeps the in-kernel grid reduction of the
    dots (its stop rule lives there), a different summation order from the
    partial sums modes 1 and 3 use: it is held to the oracle instead."""
    if case == "p2d":
        rp, cl, vl = oracle.poisson(2, 48, 40, 1)
    elif case == "p3d":
        rp, cl, vl = oracle.poisson(3, 12, 11, 10)
    else:
        rp, cl, vl = irregular_spd(20_000, seed=4)
    b = np.arange(1, len(rp), dtype=np.float64)
    out = _run_modes(rp, cl, vl, b, tol, poll=poll, graph=graph)
    x1, it1, r1 = out[1]
    for m in (3, 4):  # mode 4: p folded into the SpMV, x deferred; same values
        xm, itm, rm = out[m]
        assert itm == it1, m
        np.testing.assert_array_equal(xm, x1)
        assert rm == r1 or (np.isnan(rm) and np.isnan(r1)), (m, rm, r1)
    x2, it2, r2 = out[2]
    if tol > 0:
        xr, res = oracle.cg_solve(rp, cl, vl, b, tol)
        assert abs(it2 - res.iterations) <= max(2, res.iterations // 20)
        assert rel(x2, xr) <= (1e-10 if case != "irr" else 1e-6)
    else:   # tol 0: runs to the r.r underflow (NaN) or the N+1 cap, as mode 1
        assert np.isnan(x2).any() == np.isnan(x1).any() and it2 <= len(rp)


@pytest.mark.parametrize("mode", [2, 3, 4])
def test_fused_split_runs(queue, oracle, mode):
    """begin + several cgx_cg_run calls (each ends with the pending-x flush)
    equals one run, and the oracle capped at the same count. The splits end
    runs in every slot of mode 3's 4-body groups."""
    import ctypes as C
    from conjugategradient_amd._native import check, lib
    rp, cl, vl = oracle.poisson(2, 30, 30, 1)
    n = len(rp) - 1
    b = np.arange(1, n + 1, dtype=np.float64)
    A = Matrix(queue, vl, cl, rp)
    bv = Vector(queue, b)
    L = lib()
    xs = {}
    for split in ((23,), (5, 1, 17), (7, 16), (1, 1, 1, 1, 2, 3, 14), (4, 8, 11)):
        xv = Vector(queue, n)
        h = C.c_void_p()
        check(L.cgx_cg_create(queue.handle, A.schedule(), C.byref(h)))
        check(L.cgx_cg_set_mode(h, mode))
        check(L.cgx_cg_config(h, 4, 1))
        check(L.cgx_cg_begin(h, bv.ptr(), xv.ptr(), 0.0, 1000))
        tot, st = C.c_int64(), C.c_int()
        for k in split:
            check(L.cgx_cg_run(h, k, C.byref(tot), C.byref(st)))
        assert tot.value == 23
        xs[split] = xv.to_numpy()
        L.cgx_cg_destroy(h)
    xr, res = oracle.cg_solve(rp, cl, vl, b, 0.0, max_iter=23)
    for x in xs.values():
        np.testing.assert_array_equal(x, xs[(23,)])
    assert rel(xs[(23,)], xr) <= 1e-12


def test_large_host_copies_round_trip(queue):
    """cgx_h2d / cgx_d2h: device->host copies >= 16 MiB go through the pinned
    ring (64 MiB chunks); sizes that are not a chunk multiple, unaligned
    pointers."""
    import ctypes as C

    from conjugategradient_amd._native import check, lib
    L = lib()
    nbytes = 150 * (1 << 20) + 13
    src = np.random.default_rng(5).integers(0, 256, nbytes, dtype=np.uint8)
    d = C.c_void_p()
    check(L.cgx_alloc(queue.handle, nbytes, C.byref(d)))
    try:
        check(L.cgx_h2d(queue.handle, d, src.ctypes.data, nbytes))
        out = np.zeros(nbytes, np.uint8)
        check(L.cgx_d2h(queue.handle, out.ctypes.data, d, nbytes))
        np.testing.assert_array_equal(out, src)
        # an offset sub-range (unaligned pointers on both sides)
        part = np.zeros(nbytes - 7, np.uint8)
        check(L.cgx_d2h(queue.handle, part.ctypes.data, C.c_void_p(d.value + 7), nbytes - 7))
        np.testing.assert_array_equal(part, src[7:])
    finally:
        L.cgx_free(queue.handle, d)
