"""Matrix-Market ingest / emit (test/mm_reader.cpp read_file) through libcgx.

``read_file(path)`` returns ``(data, cols, rows)`` — the tuple order of the
reference's ``read_file`` (mm_reader.cpp:154-155), with its semantics
(include/cgx.h cgx_mm_read): the banner, line 2 always discarded, comments,
the size line, mirrored off-diagonals, (row, col) order, empty rows dropped.
The parse runs in native threads. ``write_mtx_lower`` writes the lower
triangle as a ``symmetric`` file that read_file reads back bit-identically.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._native import check, lib

__all__ = ["read_file", "write_mtx_lower"]


def read_file(path: str | os.PathLike, threads: int = 0):
    """-> (data float64[nnz], cols int32[nnz], rows int32[N+1])."""
    L = lib()
    n, nnz = C.c_int64(), C.c_int64()
    rp = C.POINTER(C.c_int32)()
    cl = C.POINTER(C.c_int32)()
    vl = C.POINTER(C.c_double)()
    check(L.cgx_mm_read(os.fsencode(path), int(threads), C.byref(n), C.byref(nnz), C.byref(rp),
                        C.byref(cl), C.byref(vl)))
    try:
        rows = np.ctypeslib.as_array(rp, shape=(n.value + 1,)).copy()
        cols = np.ctypeslib.as_array(cl, shape=(nnz.value,)).copy()
        data = np.ctypeslib.as_array(vl, shape=(nnz.value,)).copy()
    finally:
        for p in (rp, cl, vl):
            L.cgx_free_host(C.cast(p, C.c_void_p))
    return data, cols, rows


def write_mtx_lower(path: str | os.PathLike, rows, cols, data, threads: int = 0) -> None:
    """Lower triangle of a symmetric CSR as a Matrix-Market ``symmetric`` file."""
    rows = np.ascontiguousarray(rows, np.int32)
    cols = np.ascontiguousarray(cols, np.int32)
    data = np.ascontiguousarray(data, np.float64)
    check(lib().cgx_mm_write_lower(os.fsencode(path), len(rows) - 1, rows.ctypes.data,
                                   cols.ctypes.data, data.ctypes.data, int(threads)))
