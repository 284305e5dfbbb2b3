"""The setup path on the device (round 6): cgx_csr_create forms the SELL-P
plan's per-slice patterns with k_sellp_plan instead of downloading the column
array and looping over it on the host; the result must be the host plan's
(cgx_sellp_plan, the CPU suite's restatement) slot for slot. And the setup
cost is reported by phase (cgx_csr_setup_times)."""
import ctypes as C
import time

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd._native import check, lib
from tests.test_sell_cpu import sellp_plan
from tests.util import irregular_spd

pytestmark = pytest.mark.gpu


def sellp_plan_device(queue, rp, cl):
    L = lib()
    rp = np.ascontiguousarray(rp, np.int32)
    cl = np.ascontiguousarray(cl, np.int32)
    drp = cga.DeviceArray(queue, len(rp), np.int32).upload(rp)
    dcl = cga.DeviceArray(queue, max(1, len(cl)), np.int32).upload(cl)
    nsl, npat, slots, mw = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int()
    sl = C.POINTER(C.c_int64)()
    pat = C.POINTER(C.c_int32)()
    check(L.cgx_sellp_plan_device(queue.handle, drp.ptr, dcl.ptr, len(rp) - 1, len(cl),
                                  C.byref(nsl), C.byref(sl), C.byref(npat), C.byref(pat),
                                  C.byref(slots), C.byref(mw)))
    if nsl.value == 0:
        return None
    out = (np.ctypeslib.as_array(sl, shape=(nsl.value, 4)).copy(),
           np.ctypeslib.as_array(pat, shape=(npat.value,)).copy(), slots.value, mw.value)
    for p in (sl, pat):
        L.cgx_free_host(C.cast(p, C.c_void_p))
    return out


def _unsorted(rp, cl):
    cl = cl.copy()
    for i in range(len(rp) - 1):  # the first row with two entries: swap them
        if rp[i + 1] - rp[i] >= 2:
            cl[rp[i]], cl[rp[i] + 1] = cl[rp[i] + 1], cl[rp[i]]
            break
    return rp, cl


@pytest.mark.parametrize("case", ["p2d", "p3d", "p3d_ragged", "irregular", "banded_wide",
                                  "unsorted", "empty_rows", "tiny"])
def test_device_sellp_plan_is_the_host_plan(queue, oracle, case):
    if case == "p2d":
        rp, cl, _ = oracle.poisson(2, 96, 70, 1)
    elif case == "p3d":
        rp, cl, _ = oracle.poisson(3, 32, 32, 32)
    elif case == "p3d_ragged":  # n not a multiple of 128; x-lines of 7
        rp, cl, _ = oracle.poisson(3, 7, 5, 41)
    elif case == "irregular":  # the G3 stand-in's kind: too many offsets per slice
        rp, cl, _ = irregular_spd(20_000, seed=4)
    elif case == "banded_wide":  # 33 offsets per slice: one past the pattern cap
        n = 4096
        offs = np.arange(-16, 17)
        rows, cols = [], []
        for i in range(n):
            c = i + offs
            c = c[(c >= 0) & (c < n)]
            rows.append(len(c))
            cols.append(c)
        rp = np.concatenate([[0], np.cumsum(rows)]).astype(np.int32)
        cl = np.concatenate(cols).astype(np.int32)
    elif case == "unsorted":
        rp, cl = _unsorted(*oracle.poisson(2, 64, 64, 1)[:2])
    elif case == "empty_rows":  # rows without entries inside and at the end
        rp0, cl0, _ = oracle.poisson(2, 40, 40, 1)
        lens = np.diff(rp0)
        lens[100:400] = 0
        lens[-200:] = 0
        keep = np.concatenate([np.arange(rp0[i], rp0[i] + lens[i]) for i in range(len(lens))])
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        cl = cl0[keep]
    else:
        rp, cl = np.array([0, 1, 2], np.int32), np.array([0, 1], np.int32)
    host = sellp_plan(rp, cl)
    dev = sellp_plan_device(queue, rp, cl)
    if host is None:
        assert dev is None, case
        return
    assert dev is not None, case
    np.testing.assert_array_equal(dev[0], host[0])
    np.testing.assert_array_equal(dev[1], host[1])
    assert dev[2:] == host[2:]


@pytest.mark.parametrize("dim,grid", [(3, 128), (2, 1024)])
def test_setup_phases_reported(queue, dim, grid):
    """cgx_csr_setup_times: six phases whose sum is the call's wall time
    (to the host work between the marks), all non-negative."""
    L = lib()
    m = cga.Matrix.poisson(queue, dim, grid, grid, grid if dim == 3 else 1)
    queue.wait()
    h = C.c_void_p()
    t = time.perf_counter()
    check(L.cgx_csr_create(queue.handle, m.N(), m.NNZ(), m.rows().ptr, m.columns().ptr,
                           m.data().ptr, 0, None, C.byref(h)))
    wall_ms = (time.perf_counter() - t) * 1e3
    ms, cnt = (C.c_double * 6)(), C.c_int(0)
    check(L.cgx_csr_setup_times(h, ms, 6, C.byref(cnt)))
    L.cgx_csr_destroy(h)
    assert cnt.value == 6
    ph = [ms[k] for k in range(6)]
    assert all(p >= 0 for p in ph)
    assert 0.5 * wall_ms <= sum(ph) <= wall_ms * 1.01 + 1.0, (ph, wall_ms)
    assert ph[4] > 0  # the autotune ran (the matrix is past the size rule)
