"""Per-kernel timing (cgx_cg_set_kernel_timing): every timed
kernel launch takes the start / stop events its dispatch records
(hipExtLaunchKernel), the kernel's own duration as rocprofv3 reports it,
beside the event pair around the launch (dispatch latency included). bench.py
prices the roofline on the former. The timed run's x equals an untimed
(graph-replayed) run's bit for bit: the events change no kernel."""
import ctypes as C

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd._native import F64, check, lib

pytestmark = pytest.mark.gpu


def _run(L, q, A, mode, timing, bodies=24):
    n = A.N()
    b = cga.DeviceArray(q, n, np.float64)
    x = cga.DeviceArray(q, n, np.float64)
    check(L.cgx_iota(q.handle, F64, b.ptr, n, 0.0))
    x.fill(0.0)
    cg = C.c_void_p()
    check(L.cgx_cg_create(q.handle, A.schedule(), C.byref(cg)))
    try:
        check(L.cgx_cg_config(cg, 8, 1))
        check(L.cgx_cg_set_mode(cg, mode))
        check(L.cgx_cg_set_kernel_timing(cg, 1 if timing else 0))
        check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, bodies + 1))
        tot, st = C.c_int64(), C.c_int()
        check(L.cgx_cg_run(cg, bodies, C.byref(tot), C.byref(st)))
        check(L.cgx_sync(q.handle))
        d, dc = (C.c_double * 4)(), (C.c_int64 * 4)()
        e, ec = (C.c_double * 4)(), (C.c_int64 * 4)()
        check(L.cgx_cg_kernel_times(cg, d, dc))
        check(L.cgx_cg_kernel_exec_times(cg, e, ec))
        return x.download(), list(d), list(dc), list(e), list(ec)
    finally:
        L.cgx_cg_destroy(cg)


@pytest.mark.parametrize("mode", [1, 3, 4, 6])
def test_dispatch_recorded_kernel_times(queue, mode):
    L = lib()
    A = cga.Matrix.poisson(queue, 3, 128, 128, 64)
    if mode == 6:  # (Ap recomputed: the lean walk's mode; forced at this size)
        check(L.cgx_csr_set_variant(A.schedule(), 33554432))
    x_t, d, dc, e, ec = _run(L, queue, A, mode, True)
    x_g, *_ = _run(L, queue, A, mode, False)
    np.testing.assert_array_equal(x_t, x_g)
    kernels = (1, 2) if mode == 4 else (1, 2, 3)
    for k in kernels:
        # every timed launch of the body's kernels recorded its own pair
        assert dc[k] > 0 and ec[k] == dc[k], (k, dc, ec)
        # the kernel alone takes no longer than the launch around it
        assert 0.0 < e[k] <= d[k] * 1.0001, (k, d, e)
