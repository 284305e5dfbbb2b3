#!/usr/bin/env python3
"""Does the CSR-stream SpMV's time depend on where its arrays sit? The 256^3
Poisson CSR generated on the device into over-allocated buffers at chosen
byte offsets (val, col, rowptr, p, Ap), one cgx_csr per layout, variant
forced; interleaved rounds of isolated launches (cgx_tune_spmv). Prints one
JSON line per layout.

    python tools/csr_offset_probe.py [--variant 15] [--rounds 5] [--n 256]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import conjugategradient_amd as cga  # noqa: E402
from conjugategradient_amd._native import F64, check, lib  # noqa: E402

PAD = 8 << 20

# (val, col, rowptr, p, Ap) byte offsets into their allocations
LAYOUTS = {
    "aligned": (0, 0, 0, 0, 0),
    "val+4K": (4096, 0, 0, 0, 0),
    "col+4K": (0, 4096, 0, 0, 0),
    "val+64K": (65536, 0, 0, 0, 0),
    "col+1M": (0, 1 << 20, 0, 0, 0),
    "val+1M+256": (1048832, 0, 0, 0, 0),
    "p+64K": (0, 0, 0, 65536, 0),
    "all-odd": (4096 * 3, 4096 * 7, 4096 * 5, 4096 * 11, 4096 * 13),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=15)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--create", type=int, default=0,
                    help="variant forced at creation (default: --variant)")
    ap.add_argument("--layouts", default=",".join(LAYOUTS),
                    help="names from LAYOUTS, or v:c:r:p:y byte offsets (K / M suffixes)")
    a = ap.parse_args()
    os.environ["CGX_SPMV_VARIANT"] = str(a.create or a.variant)
    L = lib()
    q = cga.Queue(0)
    nx = a.n
    n = nx ** 3
    nnz = L.cgx_poisson_nnz(3, nx, nx, nx, 0, n)
    mats = {}

    def nbytes(t):
        t = t.strip()
        mul = {"K": 1024, "M": 1 << 20}.get(t[-1:], 1)
        return int(t[:-1] if mul > 1 else t) * mul

    for name in a.layouts.split(","):
        if name not in LAYOUTS:  # "v:c:r:p:y", or "v:c:r:p:y#k" for a repeat
            LAYOUTS[name] = tuple(nbytes(t) for t in name.split("#")[0].split(":"))
        ov, oc, orp, op, oy = LAYOUTS[name]
        val = cga.DeviceArray(q, nnz * 8 + PAD, np.uint8)
        col = cga.DeviceArray(q, nnz * 4 + PAD, np.uint8)
        rp = cga.DeviceArray(q, (n + 1) * 4 + PAD, np.uint8)
        p = cga.DeviceArray(q, n * 8 + PAD, np.uint8)
        y = cga.DeviceArray(q, n * 8 + PAD, np.uint8)
        check(L.cgx_poisson_fill(q.handle, F64, 3, nx, nx, nx, 0, n, rp.ptr + orp, col.ptr + oc,
                                 val.ptr + ov))
        check(L.cgx_iota(q.handle, F64, p.ptr + op, n, 1.0))
        A = C.c_void_p()
        check(L.cgx_csr_create(q.handle, n, nnz, C.c_void_p(rp.ptr + orp),
                               C.c_void_p(col.ptr + oc), C.c_void_p(val.ptr + ov), F64, None,
                               C.byref(A)))
        mats[name] = (A, (val, col, rp, p, y), (op, oy))
    times = {k: [] for k in mats}
    for _ in range(a.rounds):
        for name, (A, bufs, (op, oy)) in mats.items():
            ms = C.c_double(0)
            check(L.cgx_tune_spmv(q.handle, A, a.variant, C.c_void_p(bufs[3].ptr + op),
                                  C.c_void_p(bufs[4].ptr + oy), a.iters, C.byref(ms)))
            times[name].append(ms.value * 1e3)
    ref = None
    for name, (A, bufs, (op, oy)) in mats.items():
        out = np.empty(n)
        check(L.cgx_d2h(q.handle, out.ctypes.data, C.c_void_p(bufs[4].ptr + oy), out.nbytes))
        if ref is None:
            ref = out
        t = np.array(times[name])
        print(json.dumps({"layout": name, "offsets": LAYOUTS[name], "variant": a.variant,
                          "bases": [hex(bf.ptr) for bf in bufs],
                          "median_us": round(float(np.median(t)), 2),
                          "min_us": round(float(t.min()), 2),
                          "max_us": round(float(t.max()), 2),
                          "same_y": bool(np.array_equal(out, ref))}), flush=True)
    for A, _, _ in mats.values():
        L.cgx_csr_destroy(A)


if __name__ == "__main__":
    main()
