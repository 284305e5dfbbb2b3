"""Mode 4, the fused deferred-x iteration (cgx_abi.cpp enqueue_iter_fdefer):
two kernels per body. k_spmv_fd computes p_k = r + beta p_{k-1}
(CG.hpp:418) where the SpMV reads it and stores it into the p ring, then
helper = A p_k and its p.Ap partials (CG.hpp:374-379); update_r runs the stop
rule (CG.hpp:396-404, 436); the slot-3 flush applies the group's x updates
(CG.hpp:390). Every value is the same expression in the same order as in
modes 1 and 3, so where the fused SpMV runs on the SpMV's grid x, the body
count and the final r.r are bit-identical to mode 1 in every production SpMV
form; where it has fewer resident workgroups (big matrices) one dot's
partials split differently and x agrees to rounding. The oracle holds both."""
import ctypes as C

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd._native import check, lib
from tests.util import rel

pytestmark = pytest.mark.gpu


def _variant(m):
    v = C.c_int(0)
    check(lib().cgx_csr_variant(m.schedule(), C.byref(v)))
    return v.value


def _solve(queue, m, b, mode, tol, max_iter=-1, x0=None, poll=32):
    cg = cga.CG(queue)
    cg.mode = mode
    cg.poll_every = poll
    cg.setMatrix(m)
    cg.setTarget(b)
    if x0 is not None:
        cg.setInital(x0)
    cg.solve(tol, max_iter=max_iter)
    return cg.extract(), cg.iterations, cg.final_rxr


# (dims, grid, forced variant or None): the small-matrix rule's stencil form,
# and each production value-code form forced on a mid-size grid
CASES = [
    ("3d-rule", (3, 20, 18, 17), None),
    ("2d-rule", (2, 70, 66, 1), None),
    ("3d-stencil", (3, 64, 64, 40), 2050 | 32768 | 262144 | 524288 | 1048576),
    ("3d-pipe", (3, 64, 64, 40), 2050 | 32768 | 262144 | 524288),
    ("3d-vc8", (3, 64, 64, 40), 2050 | 32768),
    ("2d-march", (2, 1024, 640, 1), 3973122),
    ("2d-march-full", (2, 4096, 4096, 1), None),
    ("3d-full", (3, 256, 256, 256), None),
    ("3d-march", (3, 128, 128, 24), 3973122),
    ("sellp", (3, 48, 48, 30), 8194),
    # the lean walk forced (k_spmv_fd_lean: p_k formed in the gathers, the
    # formed +-D pairs carried in registers)
    ("3d-lean", (3, 128, 48, 40), "33554432:0"),
    ("csr-stream", (3, 48, 48, 30), 13),
]


@pytest.mark.parametrize("name,dims,variant", CASES, ids=[c[0] for c in CASES])
def test_mode4_bit_identical_to_mode1(queue, oracle, monkeypatch, name, dims, variant):
    if variant is not None:
        monkeypatch.setenv("CGX_SPMV_VARIANT", str(variant))
    m = cga.Matrix.poisson(queue, *dims)
    if name == "3d-lean":
        assert _variant(m) & 33554432
    n = m.N()
    gf, gs = C.c_int(), C.c_int()
    check(lib().cgx_csr_fd_grid(m.schedule(), C.byref(gf), C.byref(gs)))
    b = np.arange(1, n + 1, dtype=np.float64)  # Tester.cpp:27-30
    x1, it1, r1 = _solve(queue, m, b, 1, 0.0, max_iter=45)
    x4, it4, r4 = _solve(queue, m, b, 4, 0.0, max_iter=45)
    assert it1 == it4 == 45
    if gf.value == gs.value:  # the same p.Ap partials: every value is mode 1's
        np.testing.assert_array_equal(x4, x1)
        assert r4 == r1
    else:  # fewer resident workgroups: one dot summed in another order
        assert rel(x4, x1) <= 1e-11 and r4 == pytest.approx(r1, rel=1e-9)
    if n <= 300_000:
        rp, cl, vl = oracle.poisson(*dims)
        _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 45, 8)
        assert rel(x4, xr) <= 1e-10


def test_mode4_stop_rule_and_warm_start(queue, oracle):
    """Solve to tolerance (Q5: the body tests the r.r it started with) and a
    warm start (CG.hpp:215-219): bodies, x and the final r.r as mode 1; the
    body count lands in every slot of a 4-body group over the cases."""
    rp, cl, vl = oracle.poisson(3, 16, 15, 14)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)
    x0 = np.random.default_rng(2).standard_normal(n)
    slots = set()
    for tol in (1e-4, 1e-6, 1e-8, 1e-10):
        for start in (None, x0):
            x1, it1, r1 = _solve(queue, m, b, 1, tol * np.linalg.norm(b), x0=start)
            x4, it4, r4 = _solve(queue, m, b, 4, tol * np.linalg.norm(b), x0=start)
            assert it4 == it1
            np.testing.assert_array_equal(x4, x1)
            assert r4 == r1
            slots.add(it1 % 4)
    assert len(slots) >= 3, slots
    tol = 1e-10 * np.linalg.norm(b)
    x4, it4, _ = _solve(queue, m, b, 4, tol)
    xr, res = oracle.cg_solve(rp, cl, vl, b, tol)
    assert abs(it4 - res.iterations) <= 2 and rel(x4, xr) <= 1e-10


def test_mode4_runs_to_nan_like_mode1(queue, oracle):
    """tol 0 until r.r underflows: alpha = 0/0 turns x NaN and stops the
    loop (Q5), at the same body in both modes."""
    rp, cl, vl = oracle.poisson(2, 12, 10, 1)
    n = len(rp) - 1
    m = cga.Matrix(queue, vl, cl, rp)
    b = np.arange(1, n + 1, dtype=np.float64)
    x1, it1, _ = _solve(queue, m, b, 1, 0.0)
    x4, it4, _ = _solve(queue, m, b, 4, 0.0)
    assert it4 == it1
    assert np.isnan(x1).any() == np.isnan(x4).any()
    np.testing.assert_array_equal(np.isnan(x4), np.isnan(x1))
    np.testing.assert_array_equal(x4[~np.isnan(x4)], x1[~np.isnan(x1)])


def test_mode4_unsupported_is_refused(queue, oracle):
    rp, cl, vl = oracle.poisson(2, 10, 10, 1)
    m = cga.Matrix(queue, vl, cl, rp, dtype=np.float32)
    h = C.c_void_p()
    L = lib()
    check(L.cgx_cg_create(queue.handle, m.schedule(), C.byref(h)))
    try:
        assert L.cgx_cg_set_mode(h, 4) != 0
        assert b"mode 4" in L.cgx_last_error()
    finally:
        L.cgx_cg_destroy(h)
