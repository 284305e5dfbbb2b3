"""ctypes binding of oracle/liboracle.so and oracle/_ref/libmmref.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package. See
oracle/cg_oracle.h for what each function restates (reference file:line) and
for the parity-pinning status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libmmref.so")

_i64 = C.c_int64
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class CgResult(C.Structure):
    _fields_ = [("iterations", C.c_int64), ("rxr", C.c_double),
                ("rxr0", C.c_double), ("stopped_by_tol", C.c_int)]


def build(ref: bool = False) -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref and os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


_lib = None
_ref = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_read_mtx.argtypes = [C.c_char_p, C.POINTER(_i64), C.POINTER(_i64),
                                   C.POINTER(_ip), C.POINTER(_ip), C.POINTER(_dp)]
        L.orc_read_mtx.restype = C.c_int
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_poisson_nnz.argtypes = [C.c_int] * 4
        L.orc_poisson_nnz.restype = _i64
        L.orc_poisson.argtypes = [C.c_int] * 4 + [C.c_void_p] * 3
        L.orc_write_mtx_lower.argtypes = [C.c_char_p, _i64] + [C.c_void_p] * 3
        L.orc_write_mtx_lower.restype = C.c_int
        L.orc_spmv.argtypes = [_i64] + [C.c_void_p] * 5
        L.orc_dot_acc.argtypes = [_i64, C.c_void_p, C.c_void_p, C.c_double]
        L.orc_dot_acc.restype = C.c_double
        L.orc_norm_acc.argtypes = [_i64, C.c_void_p, C.c_double]
        L.orc_norm_acc.restype = C.c_double
        for nm in ("orc_sapbx", "orc_sambx"):
            getattr(L, nm).argtypes = [_i64, C.c_void_p, C.c_void_p, C.c_double, C.c_void_p]
        L.orc_saxpby.argtypes = [_i64, C.c_void_p, C.c_void_p, C.c_double, C.c_double,
                                 C.c_void_p]
        L.orc_cg_solve.argtypes = [_i64] + [C.c_void_p] * 5 + [C.c_int, C.c_double, _i64,
                                                               C.POINTER(CgResult)]
        L.orc_cg_solve.restype = C.c_int
        L.orc_accuracy.argtypes = [_i64] + [C.c_void_p] * 5
        L.orc_accuracy.restype = C.c_double
        L.orc_cg_fixed_iters_omp.argtypes = [_i64] + [C.c_void_p] * 5 + [_i64, C.c_int]
        L.orc_cg_fixed_iters_omp.restype = C.c_double
        L.orc_cg_timed_omp.argtypes = [_i64] + [C.c_void_p] * 5 + [_i64, _i64, C.c_int]
        L.orc_cg_timed_omp.restype = C.c_double
        L.orc_cg_solve_omp.argtypes = [_i64] + [C.c_void_p] * 5 + [C.c_int, C.c_double, _i64,
                                                                   C.c_int, C.POINTER(CgResult)]
        L.orc_cg_solve_omp.restype = C.c_int
        L.orc_cg_solve_dd.argtypes = L.orc_cg_solve_omp.argtypes
        L.orc_cg_solve_dd.restype = C.c_int
        _lib = L
    return _lib


def ref_available() -> bool:
    return os.path.exists(REF_PATH)


def ref_lib() -> C.CDLL:
    global _ref
    if _ref is None:
        L = C.CDLL(REF_PATH)
        L.mmref_read.argtypes = [C.c_char_p, C.POINTER(_i64), C.POINTER(_i64),
                                 C.POINTER(_ip), C.POINTER(_ip), C.POINTER(_dp)]
        L.mmref_read.restype = C.c_int
        L.mmref_free.argtypes = [C.c_void_p]
        _ref = L
    return _ref


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _collect(L, free, path: str):
    n, nnz = _i64(), _i64()
    rp, cl, vl = _ip(), _ip(), _dp()
    rc = L(path.encode(), C.byref(n), C.byref(nnz), C.byref(rp), C.byref(cl), C.byref(vl))
    if rc != 0:
        raise ValueError(f"read_mtx({path}) failed with code {rc}")
    rowptr = np.ctypeslib.as_array(rp, shape=(n.value + 1,)).copy()
    col = np.ctypeslib.as_array(cl, shape=(max(nnz.value, 1),))[: nnz.value].copy()
    val = np.ctypeslib.as_array(vl, shape=(max(nnz.value, 1),))[: nnz.value].copy()
    for p in (rp, cl, vl):
        free(C.cast(p, C.c_void_p))
    return rowptr, col, val


def read_mtx(path: str):
    """Restated read_file (test/mm_reader.cpp:154-171) -> (rowptr, col, val)."""
    L = lib()
    return _collect(L.orc_read_mtx, L.orc_free, path)


def ref_read_mtx(path: str):
    """The reference's own read_file, compiled from /root/reference."""
    L = ref_lib()
    return _collect(L.mmref_read, L.mmref_free, path)


def poisson(dim: int, nx: int, ny: int, nz: int = 1):
    L = lib()
    n = nx * ny * (nz if dim == 3 else 1)
    nnz = L.orc_poisson_nnz(dim, nx, ny, nz)
    rowptr = np.empty(n + 1, np.int32)
    col = np.empty(nnz, np.int32)
    val = np.empty(nnz, np.float64)
    L.orc_poisson(dim, nx, ny, nz, _ptr(rowptr), _ptr(col), _ptr(val))
    return rowptr, col, val


def write_mtx_lower(path: str, rowptr, col, val) -> None:
    rc = lib().orc_write_mtx_lower(path.encode(), len(rowptr) - 1, _ptr(rowptr), _ptr(col),
                                   _ptr(val))
    if rc:
        raise OSError(f"write_mtx_lower({path}) failed")


def spmv(rowptr, col, val, x):
    y = np.empty(len(rowptr) - 1)
    lib().orc_spmv(len(rowptr) - 1, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(x), _ptr(y))
    return y


def dot_acc(x, y, init=0.0) -> float:
    return lib().orc_dot_acc(len(x), _ptr(x), _ptr(y), init)


def norm_acc(x, init=0.0) -> float:
    return lib().orc_norm_acc(len(x), _ptr(x), init)


def sapbx(x, y, b):
    r = np.empty_like(x)
    lib().orc_sapbx(len(x), _ptr(x), _ptr(y), b, _ptr(r))
    return r


def sambx(x, y, b):
    r = np.empty_like(x)
    lib().orc_sambx(len(x), _ptr(x), _ptr(y), b, _ptr(r))
    return r


def saxpby(x, y, a, b):
    r = np.empty_like(x)
    lib().orc_saxpby(len(x), _ptr(x), _ptr(y), a, b, _ptr(r))
    return r


def cg_solve(rowptr, col, val, b, tol=0.0, x0=None, max_iter=-1):
    """Restated CG::solve (src/CG.hpp:255-454). Returns (x, CgResult)."""
    n = len(rowptr) - 1
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64, copy=True)
    res = CgResult()
    rc = lib().orc_cg_solve(n, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(b), _ptr(x),
                            0 if x0 is None else 1, tol, max_iter, C.byref(res))
    if rc:
        raise RuntimeError(f"orc_cg_solve failed: {rc}")
    return x, res


def accuracy(rowptr, col, val, b, x) -> float:
    return lib().orc_accuracy(len(rowptr) - 1, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(b),
                              _ptr(x))


def cg_fixed_iters_omp(rowptr, col, val, b, iters: int, threads: int):
    """CPU baseline: returns (seconds, x)."""
    n = len(rowptr) - 1
    x = np.zeros(n)
    t = lib().orc_cg_fixed_iters_omp(n, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(b), _ptr(x),
                                     iters, threads)
    return t, x


def cg_timed_omp(rowptr, col, val, b, warmup: int, iters: int, threads: int):
    """CPU baseline with `warmup` untimed bodies first: returns (seconds of
    the `iters` timed bodies, x)."""
    n = len(rowptr) - 1
    x = np.zeros(n)
    t = lib().orc_cg_timed_omp(n, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(b), _ptr(x),
                               warmup, iters, threads)
    return t, x


def cg_solve_omp(rowptr, col, val, b, tol: float, threads: int = 16, max_iter: int = -1,
                 x0=None):
    """orc_cg_solve on OpenMP threads: the oracle at 16.8 M rows.
    Returns (x, CgResult)."""
    n = len(rowptr) - 1
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64, copy=True)
    res = CgResult()
    rc = lib().orc_cg_solve_omp(n, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(b), _ptr(x),
                                0 if x0 is None else 1, tol, max_iter, threads, C.byref(res))
    if rc:
        raise RuntimeError(f"orc_cg_solve_omp failed: {rc}")
    return x, res


def cg_solve_dd(rowptr, col, val, b, tol: float, threads: int = 16, max_iter: int = -1, x0=None):
    """orc_cg_solve_dd: the iteration with double-length dots (the GPU
    engine's dot model; x bit for bit against it). Returns (x, CgResult)."""
    n = len(rowptr) - 1
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64, copy=True)
    res = CgResult()
    rc = lib().orc_cg_solve_dd(n, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(b), _ptr(x),
                               0 if x0 is None else 1, tol, max_iter, threads, C.byref(res))
    if rc:
        raise RuntimeError(f"orc_cg_solve_dd failed: {rc}")
    return x, res
