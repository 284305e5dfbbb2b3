#!/usr/bin/env python3
"""A/B the SpMV(+p.Ap) kernel variants on one device, interleaved rounds in
one process (cdna_hip_programming.md §5.4 rule 24). Prints one JSON line per
(config, variant): median/min us and algorithmic GB/s; checks every variant's
y against variant 0 bit for bit.

    python tools/tune_spmv.py [--configs 3d256,2d4096,irr] [--rounds 5] [--iters 20]
                              [--orders 0,-1,2048]   (CSR-stream block orders,
                              cgx_csr_set_block_order's chunk rows)
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
from conjugategradient_amd._native import check, lib  # noqa: E402


def matrix(q, name):
    if name == "3d256":
        return cga.Matrix.poisson(q, 3, 256, 256, 256)
    if name == "3d128":
        return cga.Matrix.poisson(q, 3, 128, 128, 128)
    if name == "2d4096":
        return cga.Matrix.poisson(q, 2, 4096, 4096, 1)
    if name.startswith("g2:") or name.startswith("g3:"):  # g3:NXxNYxNZ, g2:NXxNY
        dims = [int(v) for v in name[3:].split("x")]
        return cga.Matrix.poisson(q, int(name[1]), *dims)
    if name == "irr":
        from tests.util import irregular_spd
        rp, cl, vl = irregular_spd(1_585_478, mean_deg=3.83, seed=12345)
        return cga.Matrix(q, vl, cl, rp)
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="3d256,2d4096,irr")
    ap.add_argument("--variants", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--orders", default="")
    a = ap.parse_args()
    L = lib()
    q = cga.Queue(0)
    variants = [int(v) for v in a.variants.split(",")]
    orders = [int(o) for o in a.orders.split(",")] if a.orders else [None]
    if any(v & 2048 for v in variants):  # keep the SELL-64 copy (autotune may free it)
        os.environ.setdefault("CGX_SPMV_VARIANT", "2048")
    for name in a.configs.split(","):
        A = matrix(q, name)
        n, nnz = A.N(), A.NNZ()
        if any(v & 67108864 for v in variants):  # build the interleaved val / col copy (kIL)
            check(L.cgx_csr_set_variant(A.schedule(), 67108879))
        # a second schedule with half tiles for the variants with bit 64
        half = C.c_void_p()
        check(L.cgx_csr_create(q.handle, n, nnz, A.rows().ptr, A.columns().ptr, A.data().ptr, 0,
                               None, C.byref(half)))
        check(L.cgx_csr_set_tile(half, 1024))
        wave = C.c_void_p()  # wave tiles for the variants with bit 512
        check(L.cgx_csr_create(q.handle, n, nnz, A.rows().ptr, A.columns().ptr, A.data().ptr, 0,
                               None, C.byref(wave)))
        check(L.cgx_csr_set_tile(wave, 512))
        pair = None  # SELL with 2 rows per lane for the variants with bit 4096
        if any(v & 4096 for v in variants):
            pair = C.c_void_p()
            check(L.cgx_csr_create(q.handle, n, nnz, A.rows().ptr, A.columns().ptr,
                                   A.data().ptr, 0, None, C.byref(pair)))
            check(L.cgx_csr_set_sell(pair, 2))
        x = cga.Vector(q, np.random.default_rng(0).standard_normal(n))
        keys = [(v, o) for v in variants for o in orders]
        ys = {k: cga.Vector(q, n) for k in keys}
        times = {k: [] for k in keys}
        used = {}
        for _ in range(a.rounds):
            for v, o in keys:
                ms = C.c_double(0)
                sched = (pair if v & 4096 else wave if v & 512 else half if v & 64
                         else A.schedule())
                if o is not None:
                    check(L.cgx_csr_set_block_order(sched, o))
                    d, w = C.c_int(), C.c_int()
                    check(L.cgx_csr_block_order_info(sched, C.byref(d), C.byref(w)))
                    used[(v, o)] = [d.value, w.value]
                check(L.cgx_tune_spmv(q.handle, sched, v, x.ptr(), ys[(v, o)].ptr(), a.iters,
                                      C.byref(ms)))
                times[(v, o)].append(ms.value)
        y0 = ys[keys[0]].to_numpy()
        nbytes = 12 * nnz + 4 * (n + 1) + 16 * n
        for v, o in keys:
            t = np.array(times[(v, o)]) * 1e3
            same = bool(np.array_equal(ys[(v, o)].to_numpy(), y0))
            print(json.dumps({"config": name, "variant": v, "order": used.get((v, o)),
                              "n": n, "nnz": nnz,
                              "median_us": round(float(np.median(t)), 2),
                              "min_us": round(float(t.min()), 2),
                              "GBps_median": round(nbytes / (np.median(t) * 1e-6) / 1e9, 1),
                              "bitexact_vs_v0": same}), flush=True)
        L.cgx_csr_destroy(half)
        L.cgx_csr_destroy(wave)
        if pair is not None:
            L.cgx_csr_destroy(pair)
        del A, x, ys


if __name__ == "__main__":
    main()
