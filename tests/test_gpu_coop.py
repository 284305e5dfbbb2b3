"""Mode 5, the persistent body (cgx_coop.hip): one launch runs a chunk of
loop bodies of CG::solve (CG.hpp:359-436), each with two grid-wide exchanges
of the dot partials instead of three kernel boundaries. The SpMV is the
reference's per-row loop (VectorOperations.hpp:456-459), so Ap is bit-exact;
the dots are summed in another order than in modes 1-4, so x agrees with the
oracle to rounding (rel <= 1e-10) and the body count within 2 at a
tolerance; the stop rule is the reference's (CG.hpp:396-404, 436)."""
import ctypes as C

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd._native import check, lib
from tests.util import irregular_spd, rel

pytestmark = pytest.mark.gpu


def _shape(h):
    """(rows per thread, threads, workgroups, form) of a mode-5 solver"""
    v = [C.c_int() for _ in range(4)]
    check(lib().cgx_cg_coop_shape(h, *[C.byref(a) for a in v]))
    return tuple(a.value for a in v)


def _solve(queue, m, b, mode, tol, max_iter=-1, x0=None, poll=32, shape=None):
    cg = cga.CG(queue)
    cg.mode = mode
    cg.poll_every = poll
    cg.setMatrix(m)
    cg.setTarget(b)
    if x0 is not None:
        cg.setInital(x0)
    cg.solve(tol, max_iter=max_iter)
    if shape is not None:
        shape.append(_shape(cg._cg))
    return cg.extract(), cg.iterations, cg.final_rxr


@pytest.mark.parametrize("dims", [(2, 128, 128, 1), (3, 20, 18, 17), (2, 70, 66, 1)],
                         ids=["p2d_128", "p3d_20x18x17", "p2d_70x66"])
def test_mode5_fixed_bodies_match_oracle(queue, oracle, dims):
    """the register form (one row per thread of 1,024)"""
    rp, cl, vl = oracle.poisson(*dims)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)  # Tester.cpp:27-30
    x5, it5, r5 = _solve(queue, m, b, 5, 0.0, max_iter=45)
    x1, it1, r1 = _solve(queue, m, b, 1, 0.0, max_iter=45)
    assert it5 == it1 == 45
    assert rel(x5, x1) <= 1e-11 and r5 == pytest.approx(r1, rel=1e-9)
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 45, 8)
    assert rel(x5, xr) <= 1e-10


@pytest.mark.parametrize("R", ["1", "2", "3"])
@pytest.mark.parametrize("dims", [(2, 128, 128, 1), (3, 20, 18, 17), (2, 70, 66, 1)],
                         ids=["p2d_128", "p3d_20x18x17", "p2d_70x66"])
def test_mode5_streamed_fixed_bodies_match_oracle(queue, oracle, monkeypatch, dims, R):
    """The streamed form ($CGX_COOP_STREAM=1): R rows per thread of 1,024,
    the matrix's entries staged through LDS chunk by chunk."""
    monkeypatch.setenv("CGX_COOP_STREAM", "1")
    monkeypatch.setenv("CGX_COOP_R", R)
    rp, cl, vl = oracle.poisson(*dims)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)
    shape = []
    x5, it5, r5 = _solve(queue, m, b, 5, 0.0, max_iter=45, shape=shape)
    assert shape[0][0] == int(R) and shape[0][1] == 1024 and shape[0][3] == 2
    assert shape[0][2] == -(-n // (1024 * int(R)))
    x1, it1, r1 = _solve(queue, m, b, 1, 0.0, max_iter=45)
    assert it5 == it1 == 45
    assert rel(x5, x1) <= 1e-11 and r5 == pytest.approx(r1, rel=1e-9)
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 45, 8)
    assert rel(x5, xr) <= 1e-10


def test_mode5_streamed_long_rows_and_tolerance(queue, oracle, monkeypatch):
    """A chunk with more entries than the LDS stage (a hub row of 30,000
    entries) is summed from the CSR arrays; to tolerance and warm, with the
    stop inside and at the end of launches."""
    monkeypatch.setenv("CGX_COOP_STREAM", "1")
    rp, cl, vl = irregular_spd(40000, seed=4, hub=30000, shift=10.0)
    assert np.diff(rp).max() > 20000
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, len(rp), dtype=np.float64)
    x5, it5, _ = _solve(queue, m, b, 5, 0.0, max_iter=30)
    assert it5 == 30
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 30, 8)
    assert rel(x5, xr) <= 1e-10
    rp, cl, vl = oracle.poisson(3, 16, 15, 14)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)
    x0 = np.random.default_rng(2).standard_normal(n)
    for start in (None, x0):
        for poll in (1, 32):
            t = 1e-8 * np.linalg.norm(b)
            x5, it5, _ = _solve(queue, m, b, 5, t, x0=start, poll=poll)
            x1, it1, _ = _solve(queue, m, b, 1, t, x0=start)
            assert abs(it5 - it1) <= 2 and rel(x5, x1) <= 1e-9


def test_mode5_streamed_g3_standin(queue, oracle, monkeypatch):
    """The G3_circuit stand-in (1,585,478 rows) in the streamed
    form: 7 rows per thread, 222 workgroups; 20 bodies against mode 3."""
    from conjugategradient_amd import workloads
    monkeypatch.setenv("CGX_COOP_STREAM", "1")
    rp, cl, vl = workloads.host_csr("g3_standin")
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, len(rp), dtype=np.float64)
    shape = []
    x5, it5, r5 = _solve(queue, m, b, 5, 0.0, max_iter=20, shape=shape)
    assert shape[0][3] == 2
    x3, it3, r3 = _solve(queue, m, b, 3, 0.0, max_iter=20)
    assert it5 == it3 == 20
    print("g3 streamed vs mode 3: rel", rel(x5, x3), "shape", shape[0])
    assert rel(x5, x3) <= 1e-8


def test_mode5_solves_to_tolerance_and_warm_start(queue, oracle):
    """To tolerance, cold and warm (CG.hpp:215-219), with chunks of 8 bodies
    per launch (poll 1): the stop lands inside and at the end of launches."""
    rp, cl, vl = oracle.poisson(3, 16, 15, 14)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)
    x0 = np.random.default_rng(2).standard_normal(n)
    for tol in (1e-4, 1e-8, 1e-10):
        for start in (None, x0):
            for poll in (1, 32):
                t = tol * np.linalg.norm(b)
                x5, it5, r5 = _solve(queue, m, b, 5, t, x0=start, poll=poll)
                x1, it1, r1 = _solve(queue, m, b, 1, t, x0=start)
                assert abs(it5 - it1) <= 2, (tol, poll, it5, it1)
                assert rel(x5, x1) <= 1e-9
    t = 1e-10 * np.linalg.norm(b)
    x5, it5, _ = _solve(queue, m, b, 5, t)
    xr, res = oracle.cg_solve(rp, cl, vl, b, t)
    assert abs(it5 - res.iterations) <= 2 and rel(x5, xr) <= 1e-10


def test_mode5_register_form_on_256_workgroups(queue, oracle):
    """512^2 (262,144 rows): the register form on 256 workgroups of 1,024
    threads, one per CU (the exchange sweep reads four partials per lane)."""
    rp, cl, vl = oracle.poisson(2, 512, 512, 1)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)
    shape = []
    x5, it5, r5 = _solve(queue, m, b, 5, 0.0, max_iter=40, shape=shape)
    assert shape[0] == (1, 1024, 256, 0)
    x1, it1, r1 = _solve(queue, m, b, 1, 0.0, max_iter=40)
    assert it5 == it1 == 40
    assert rel(x5, x1) <= 1e-11 and r5 == pytest.approx(r1, rel=1e-9)


@pytest.mark.parametrize("stream", ["0", "1"], ids=["register", "streamed"])
def test_mode5_irregular_rows(queue, oracle, monkeypatch, stream):
    """Rows longer than the kCoopK entries held in registers (a hub row of
    300 entries) read their tail from the CSR arrays. Diagonal shift 10: a
    well-conditioned system, where 30 bodies in two summation orders agree to
    1e-15 on the CPU (with the stand-in's shift of 1e-2 the oracle's own 1-
    and 8-thread runs differ by 5e-3 after 30 bodies on this hub matrix)."""
    monkeypatch.setenv("CGX_COOP_STREAM", stream)
    rp, cl, vl = irregular_spd(20000, seed=4, hub=300, shift=10.0)
    assert np.diff(rp).max() > 8
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, len(rp), dtype=np.float64)
    x5, it5, _ = _solve(queue, m, b, 5, 0.0, max_iter=30)
    assert it5 == 30
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 30, 8)
    assert rel(x5, xr) <= 1e-10


def test_mode5_runs_to_nan_like_mode1(queue, oracle):
    rp, cl, vl = oracle.poisson(2, 12, 10, 1)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)
    x5, it5, _ = _solve(queue, m, b, 5, 0.0)
    # tol 0 runs until r.r is exactly 0 (alpha = 0/0 turns x NaN and the NaN
    # rule stops at the next body, Q5) or to the cap of N + 1 bodies; which
    # body that is depends on the dots' rounding
    assert it5 <= n + 1
    if np.isnan(x5).any():
        assert it5 < n + 1


def test_mode5_refused_where_it_does_not_apply(queue, oracle):
    L = lib()
    rp, cl, vl = oracle.poisson(2, 10, 10, 1)
    m = cga.Matrix(queue, vl, cl, rp, dtype=np.float32)
    h = C.c_void_p()
    check(L.cgx_cg_create(queue.handle, m.schedule(), C.byref(h)))
    try:
        assert L.cgx_cg_set_mode(h, 5) != 0
        assert b"mode 5" in L.cgx_last_error()
    finally:
        L.cgx_cg_destroy(h)
    # past the streamed form: 8 rows x 1,024 threads x 256 workgroups
    big = cga.Matrix.poisson(queue, 3, 130, 130, 130)  # 2,197,000 rows
    check(L.cgx_cg_create(queue.handle, big.schedule(), C.byref(h)))
    try:
        assert L.cgx_cg_set_mode(h, 5) != 0
        assert b"at most" in L.cgx_last_error()
    finally:
        L.cgx_cg_destroy(h)
    del big
    # which form: a 3-D stencil of 163,840 rows (160 workgroups) keeps its
    # entries in registers, also in auto; an irregular 200k-row matrix (rows
    # past 7 entries) takes the streamed form, also in auto (CSR-stream path,
    # one row per thread); 1,000,000 rows: the streamed form only when asked
    rp, cl, vl = irregular_spd(200000, seed=5)
    cases = ((lambda: cga.Matrix.poisson(queue, 3, 64, 64, 40), True, 0),
             (lambda: cga.Matrix(queue, vl, cl, rp), True, 2),
             (lambda: cga.Matrix.poisson(queue, 3, 100, 100, 100), False, 2))
    for make, auto5, form in cases:
        mid = make()
        check(L.cgx_cg_create(queue.handle, mid.schedule(), C.byref(h)))
        try:
            check(L.cgx_cg_set_mode(h, 0))
            mode = C.c_int()
            check(L.cgx_cg_get_mode(h, C.byref(mode)))
            assert (mode.value == 5) == auto5
            check(L.cgx_cg_set_mode(h, 5))
            assert _shape(h)[3] == form
        finally:
            L.cgx_cg_destroy(h)


@pytest.mark.parametrize("stream", ["0", "1"])
def test_mode5_stalled_exchange_times_out_and_recovers(queue, oracle, monkeypatch, stream):
    """Every spin of the persistent body is bounded: with workgroup 0
    withholding one body's p.Ap partial (fault injection), the others give
    up after $CGX_COOP_TIMEOUT_MS and raise the shared flag, the launch ends,
    cgx_cg_run reports it (stopped = 4), and the device and a new solver
    work normally afterwards."""
    rp, cl, vl = oracle.poisson(2, 64, 64, 1)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)
    monkeypatch.setenv("CGX_COOP_STREAM", stream)
    monkeypatch.setenv("CGX_COOP_INJECT_STALL", "3")
    monkeypatch.setenv("CGX_COOP_TIMEOUT_MS", "50")
    with pytest.raises(Exception, match="mode 5"):
        _solve(queue, m, b, 5, 0.0, max_iter=20)
    monkeypatch.delenv("CGX_COOP_INJECT_STALL")
    monkeypatch.delenv("CGX_COOP_TIMEOUT_MS")
    x5, it5, _ = _solve(queue, m, b, 5, 0.0, max_iter=20)
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 20, 8)
    assert it5 == 20 and rel(x5, xr) <= 1e-10
