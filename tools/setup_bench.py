#!/usr/bin/env python3
"""Setup-path timings: host->device upload of a 256^3
CSR (1.47 GB) through the pinned ring vs a single hipMemcpy, download, and
cgx_csr_create (row-block schedule + SELL copy + SpMV autotune).

    python tools/setup_bench.py [--grid 256]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import conjugategradient_amd as cga  # noqa: E402
from conjugategradient_amd._native import check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--dim", type=int, default=3)
    a = ap.parse_args()
    L = lib()
    q = cga.Queue(0)
    m = cga.Matrix.poisson(q, a.dim, a.grid, a.grid, a.grid if a.dim == 3 else 1)
    rows, cols, data = m.rows().download(), m.columns().download(), m.data().download()
    nbytes = rows.nbytes + cols.nbytes + data.nbytes
    out = {"grid": a.grid, "csr_bytes": nbytes}
    for rep in ("a", "b"):
        t = time.perf_counter()
        A = cga.Matrix(q, data, cols, rows)
        dt = time.perf_counter() - t
        out.setdefault("h2d_GBps", []).append(round(nbytes / dt / 1e9, 2))
        t = time.perf_counter()
        A.data().download()
        dt = time.perf_counter() - t
        out.setdefault("d2h_GBps", []).append(round(data.nbytes / dt / 1e9, 2))
        del A
    # cgx_csr_create by phase, against a solve to 1e-8 ||b|| on the same matrix
    # (verdict r5 item 8: setup vs. the solve it serves)
    ms, cnt = (C.c_double * 6)(), C.c_int(0)
    for rep in range(2):
        q.wait()
        t = time.perf_counter()
        h = C.c_void_p()
        check(L.cgx_csr_create(q.handle, m.N(), m.NNZ(), m.rows().ptr, m.columns().ptr,
                               m.data().ptr, 0, None, C.byref(h)))
        q.wait()
        out.setdefault("csr_create_s", []).append(round(time.perf_counter() - t, 4))
        check(L.cgx_csr_setup_times(h, ms, 6, C.byref(cnt)))
        out.setdefault("phases_ms", []).append([round(ms[k], 1) for k in range(6)])
        if rep == 1:
            n = m.N()
            b = cga.DeviceArray(q, n, np.float64)
            x = cga.DeviceArray(q, n, np.float64)
            check(L.cgx_iota(q.handle, 0, b.ptr, n, 0.0))
            bn = float(np.linalg.norm(np.arange(1, n + 1, dtype=np.float64)))
            cg = C.c_void_p()
            check(L.cgx_cg_create(q.handle, h, C.byref(cg)))
            for k in range(2):  # the first one captures the graphs
                x.fill(0.0)
                q.wait()
                t = time.perf_counter()
                it, rr = C.c_int64(), C.c_double()
                check(L.cgx_cg_solve(cg, b.ptr, x.ptr, 1e-8 * bn, -1, C.byref(it), C.byref(rr)))
                q.wait()
                out.setdefault("solve_1e-8_s", []).append(round(time.perf_counter() - t, 4))
            out["solve_bodies"] = it.value
            L.cgx_cg_destroy(cg)
        L.cgx_csr_destroy(h)
    out["phase_names"] = ["schedule", "sell_plan_pack", "value_codes", "split", "autotune", "rest"]
    for sell in ("0", "3"):
        t = time.perf_counter()
        h = C.c_void_p()
        check(L.cgx_csr_create(q.handle, m.N(), m.NNZ(), m.rows().ptr, m.columns().ptr,
                               m.data().ptr, 0, rows.ctypes.data, C.byref(h)))
        if sell == "0":  # the CSR-stream schedule alone: the SELL copy dropped again
            check(L.cgx_csr_set_sell(h, 0))
        out[f"csr_create_s_sell{sell}"] = round(time.perf_counter() - t, 3)
        v = C.c_int()
        check(L.cgx_csr_variant(h, C.byref(v)))
        out[f"variant_sell{sell}"] = v.value
        L.cgx_csr_destroy(h)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
