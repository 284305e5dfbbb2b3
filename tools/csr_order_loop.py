#!/usr/bin/env python3
"""CSR-stream's block visit order inside the CG loop: the same matrix in one
CSR-stream variant with each requested order (cgx_csr_set_block_order's
chunk rows; 0 natural, -1 automatic), interleaved rounds in one process.
Prints per (order, round) the iterations/s over graph-replayed bodies and
the SpMV's HIP-event time.

    python tools/csr_order_loop.py [--grid 256] [--variant 15] [--orders 0,-1] [--rounds 2]
"""
from __future__ import annotations

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
from conjugategradient_amd._native import F64, check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--variant", type=int, default=15)
    ap.add_argument("--orders", default="0,-1")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--bodies", type=int, default=60)
    ap.add_argument("--mode", type=int, default=3)
    a = ap.parse_args()
    L = lib()
    q = cga.Queue(0)
    g = a.grid
    A = cga.Matrix.poisson(q, 3, g, g, g)
    n, nnz = A.N(), A.NNZ()
    sched = A.schedule()
    check(L.cgx_csr_set_variant(sched, a.variant))
    b = cga.DeviceArray(q, n, np.float64)
    x = cga.DeviceArray(q, n, np.float64)
    check(L.cgx_iota(q.handle, F64, b.ptr, n, 0.0))
    csr_bytes = 12 * nnz + 4 * (n + 1) + 16 * n
    for rnd in range(a.rounds):
        for o in (int(v) for v in a.orders.split(",")):
            check(L.cgx_csr_set_block_order(sched, o))
            d, w = C.c_int(), C.c_int()
            check(L.cgx_csr_block_order_info(sched, C.byref(d), C.byref(w)))
            x.fill(0.0)
            cg = C.c_void_p()
            check(L.cgx_cg_create(q.handle, sched, C.byref(cg)))
            check(L.cgx_cg_config(cg, 64, 1))
            check(L.cgx_cg_set_mode(cg, a.mode))
            check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, 10 + a.bodies + 1))
            tot, st = C.c_int64(), C.c_int()
            check(L.cgx_cg_run(cg, 10, C.byref(tot), C.byref(st)))
            check(L.cgx_sync(q.handle))
            t = time.perf_counter()
            check(L.cgx_cg_run(cg, a.bodies, C.byref(tot), C.byref(st)))
            check(L.cgx_sync(q.handle))
            dt = time.perf_counter() - t
            avg = (C.c_double * 4)()
            calls = (C.c_int64 * 4)()
            check(L.cgx_cg_set_kernel_timing(cg, 1))
            check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, 41))
            check(L.cgx_cg_run(cg, 40, C.byref(tot), C.byref(st)))
            check(L.cgx_cg_kernel_times(cg, avg, calls))
            L.cgx_cg_destroy(cg)
            spmv_us = avg[1] * 1e3
            print(json.dumps({"round": rnd, "order": [d.value, w.value], "variant": a.variant,
                              "it_per_s": round(a.bodies / dt, 1),
                              "spmv_us": round(spmv_us, 2),
                              "spmv_csr_frac": round(csr_bytes / (spmv_us * 1e-6) / 8e12, 4),
                              "update_r_us": round(avg[2] * 1e3, 2),
                              "p_update_us": round(avg[3] * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
