"""libcgx.so on a CPU-only host: it loads, exports every entry point
include/cgx.h declares, its host-only helpers are right, and compute entry
points fail loudly (no silent fallback) when there is no device."""
import ctypes as C
import os

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd._native import CgxError, lib

ON_GPU_HOST = os.path.exists("/dev/kfd")


def test_all_header_symbols_exported():
    L = lib()
    syms = cga.header_symbols()
    assert len(syms) >= 40
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_version_and_device_count():
    assert lib().cgx_version().startswith(b"cgx")
    assert cga.device_count() >= 0


@pytest.mark.skipif(ON_GPU_HOST, reason="checks the no-device failure path")
def test_no_device_fails_loudly():
    with pytest.raises(CgxError, match="device|ROCm"):
        cga.Queue(0)
    with pytest.raises(CgxError):
        cga.CG.createCG()


@pytest.mark.parametrize("dim,nx,ny,nz", [(2, 16, 16, 1), (3, 16, 16, 16), (3, 7, 5, 3),
                                          (2, 1, 9, 1), (3, 256, 256, 256)])
def test_poisson_nnz_formula(oracle, dim, nx, ny, nz):
    L = lib()
    n = nx * ny * (nz if dim == 3 else 1)
    assert L.cgx_poisson_nnz(dim, nx, ny, nz, 0, n) == oracle.lib().orc_poisson_nnz(dim, nx, ny,
                                                                                    nz)
    if n <= 5000:
        rp, _, _ = oracle.poisson(dim, nx, ny, nz)
        for a in range(0, n + 1, max(1, n // 37)):
            for b in (a, min(n, a + 13), n):
                assert L.cgx_poisson_nnz(dim, nx, ny, nz, a, b) == rp[b] - rp[a]


def _row_blocks(rowptr):
    L = lib()
    nrb = C.c_int64()
    ptr = C.POINTER(C.c_int)()
    mx = C.c_int()
    rc = L.cgx_row_blocks(rowptr.ctypes.data, len(rowptr) - 1, C.byref(nrb), C.byref(ptr),
                          C.byref(mx))
    assert rc == 0
    rb = np.ctypeslib.as_array(ptr, shape=(nrb.value + 1,)).copy()
    L.cgx_free_host(C.cast(ptr, C.c_void_p))
    return rb, mx.value


@pytest.mark.parametrize("case", ["poisson", "irregular", "hub", "empty_rows"])
def test_row_block_schedule(oracle, case):
    from tests.util import irregular_spd

    if case == "poisson":
        rp, _, _ = oracle.poisson(3, 20, 20, 20)
    elif case == "irregular":
        rp, _, _ = irregular_spd(30_000, seed=2)
    elif case == "hub":
        rp, _, _ = irregular_spd(10_000, seed=2, hub=4000)
    else:
        rp = np.array([0, 0, 0, 3, 3, 5, 5], np.int32)
    rb, mx = _row_blocks(rp)
    n = len(rp) - 1
    assert rb[0] == 0 and rb[-1] == n and np.all(np.diff(rb) >= 1)
    assert mx == np.diff(rp).max()
    for a, b in zip(rb[:-1], rb[1:]):
        cnt = rp[b] - rp[a]
        assert b - a <= 256
        assert cnt <= 2042 or b - a == 1      # a long row is alone
    if case == "poisson":
        assert np.all(np.diff(rb)[:-1] == 256)  # 7-nnz rows fill whole blocks


def test_halo_plan_helpers(oracle):
    """cgx_plan_ghosts / cgx_plan_remap on a 3-rank z-slab split."""
    L = lib()
    nx = ny = 6
    nz = 9
    rp, cl, vl = oracle.poisson(3, nx, ny, nz)
    n = len(rp) - 1
    world = 3
    begins = np.array([0, n // 3, 2 * n // 3], np.int64)
    counts = np.array([n // 3, n // 3, n - 2 * (n // 3)], np.int64)
    for r in range(world):
        a, b = begins[r], begins[r] + counts[r]
        lcol = cl[rp[a]:rp[b]].copy()
        ng = C.c_int64()
        gp = C.POINTER(C.c_int64)()
        recv = np.zeros(world, np.int64)
        assert L.cgx_plan_ghosts(counts[r], a, len(lcol), lcol.ctypes.data, world,
                                 begins.ctypes.data, counts.ctypes.data, C.byref(ng),
                                 C.byref(gp), recv.ctypes.data) == 0
        ghosts = np.ctypeslib.as_array(gp, shape=(max(ng.value, 1),))[:ng.value].copy()
        want = np.unique(lcol[(lcol < a) | (lcol >= b)])
        np.testing.assert_array_equal(ghosts, want)
        plane = nx * ny
        assert recv[r] == 0
        assert recv.sum() == ng.value == plane * ((r > 0) + (r < world - 1))
        assert L.cgx_plan_remap(counts[r], a, len(lcol), lcol.ctypes.data, ng.value,
                                gp) == 0
        # local numbering maps back to the global columns
        back = np.where(lcol < counts[r], lcol + a, ghosts[np.maximum(lcol - counts[r], 0)])
        np.testing.assert_array_equal(back, cl[rp[a]:rp[b]])
        L.cgx_free_host(C.cast(gp, C.c_void_p))
    # ranges out of rank order are rejected
    bad = np.array([n // 2, 0], np.int64)
    cnt2 = np.array([n - n // 2, n // 2], np.int64)
    lcol = cl[:rp[n // 2]].copy()
    ng = C.c_int64()
    gp = C.POINTER(C.c_int64)()
    recv = np.zeros(2, np.int64)
    assert L.cgx_plan_ghosts(n // 2, 0, len(lcol), lcol.ctypes.data, 2, bad.ctypes.data,
                             cnt2.ctypes.data, C.byref(ng), C.byref(gp), recv.ctypes.data) != 0
