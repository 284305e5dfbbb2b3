"""Handle lifetimes through the raw C ABI (include/cgx.h): libcgx refcounts a
context from the matrices and solvers made on it, and a matrix from its
solvers, so any destruction order is valid — the owner's cgx_destroy /
cgx_csr_destroy only drops the owner's reference. A solver still runs after
its context's and matrix's owners let go, and gives the same x."""
import ctypes as C

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd._native import F64, check, lib

pytestmark = pytest.mark.gpu


def _setup(n2=24):
    L = lib()
    ctx = C.c_void_p()
    check(L.cgx_create(0, C.byref(ctx)))
    n = n2 * n2
    nnz = L.cgx_poisson_nnz(2, n2, n2, 1, 0, n)
    bufs = {}
    for name, count, es in (("rows", n + 1, 4), ("cols", nnz, 4), ("vals", nnz, 8), ("b", n, 8),
                            ("x", n, 8)):
        p = C.c_void_p()
        check(L.cgx_alloc(ctx, count * es, C.byref(p)))
        bufs[name] = p
    check(L.cgx_poisson_fill(ctx, F64, 2, n2, n2, 1, 0, n, bufs["rows"], bufs["cols"],
                             bufs["vals"]))
    check(L.cgx_iota(ctx, F64, bufs["b"], n, 0.0))
    check(L.cgx_fill(ctx, F64, bufs["x"], 0.0, n))
    A = C.c_void_p()
    check(L.cgx_csr_create(ctx, n, nnz, bufs["rows"], bufs["cols"], bufs["vals"], F64, None,
                           C.byref(A)))
    cg = C.c_void_p()
    check(L.cgx_cg_create(ctx, A, C.byref(cg)))
    return L, ctx, A, cg, bufs, n


def _solve(L, cg, bufs, n):
    bodies, rxr = C.c_int64(), C.c_double()
    check(L.cgx_cg_solve(cg, bufs["b"], bufs["x"], 1e-8, -1, C.byref(bodies), C.byref(rxr)))
    return bodies.value


def test_destroy_context_and_matrix_before_solver():
    L, ctx, A, cg, bufs, n = _setup()
    # device buffers are plain hipMalloc memory, freed by the caller: keep
    # them; let go of the context's and the matrix's owner references first
    ref = _setup()
    it_ref = _solve(ref[0], ref[3], ref[4], ref[5])
    x_ref = np.empty(n)
    check(L.cgx_d2h(ref[1], x_ref.ctypes.data, ref[4]["x"], n * 8))
    check(L.cgx_csr_destroy(A))   # the solver still holds the matrix
    check(L.cgx_destroy(ctx))     # ... and the context
    it = _solve(L, cg, bufs, n)   # runs on the released-by-owner objects
    x = np.empty(n)
    # the context is still alive: the solver's reference keeps it
    check(L.cgx_d2h(ctx, x.ctypes.data, bufs["x"], n * 8))
    assert it == it_ref
    np.testing.assert_array_equal(x, x_ref)
    check(L.cgx_cg_destroy(cg))   # last reference: matrix, then context freed
    for name in bufs:  # plain device memory of the same device
        check(L.cgx_free(ref[1], bufs[name]))
        check(L.cgx_free(ref[1], ref[4][name]))
    check(ref[0].cgx_cg_destroy(ref[3]))
    check(ref[0].cgx_csr_destroy(ref[2]))
    check(ref[0].cgx_destroy(ref[1]))


def test_python_objects_outlive_closed_queue():
    q = cga.Queue(0)
    cg = cga.CG(q)
    cg.setMatrix(cga.Matrix.poisson(q, 2, 16, 16))
    cg.setTarget(np.arange(1, 257, dtype=np.float64))
    cg.solve(1e-8)
    q.close()  # the owner's reference goes; matrix and solver keep theirs
    cg._drop_solver()
    cg.A._drop_schedule()
