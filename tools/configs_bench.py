#!/usr/bin/env python3
"""CG iteration throughput on the SURVEY §8(d) configurations, one GPU:

  p2d_128   128^2 Poisson read from tests/golden/poisson2d_128.mtx (cga.read_file)
  p2d_4096  4096^2 Poisson (device generator)
  p3d_256   256^3 Poisson (the bench.py workload)
  p3d_512   512^3 Poisson on one GPU (the 8-GPU strong-scaling problem)
  g3_irr    the G3_circuit stand-in: seeded irregular SPD, N = 1,585,478

Each config: b_i = i + 1, x0 = 0, tol 0 with a body cap, W warm-up bodies,
then K timed bodies (one cgx_cg_run, graph replay, bracketed by syncs).
Prints one JSON line per config: it/s, B_alg GB/s (12 nnz + 4 (N+1) + 80 N
per iteration), fraction of 8 TB/s, the SpMV variant.

    python tools/configs_bench.py [--configs p2d_128,p2d_4096,p3d_256,p3d_512,g3_irr]
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

PEAK = 8000.0
# (steps, warmup)
PLAN = {"p2d_128": (600, 20), "p2d_4096": (400, 20), "p3d_256": (400, 20),
        "p3d_512": (80, 5), "g3_irr": (2000, 50)}


def matrix(q, name):
    if name == "p2d_128":
        data, cols, rows = cga.read_file(os.path.join(ROOT, "tests", "golden",
                                                      "poisson2d_128.mtx"))
        return cga.Matrix(q, data, cols, rows)
    if name == "p2d_4096":
        return cga.Matrix.poisson(q, 2, 4096, 4096, 1)
    if name == "p3d_256":
        return cga.Matrix.poisson(q, 3, 256, 256, 256)
    if name == "p3d_512":
        return cga.Matrix.poisson(q, 3, 512, 512, 512)
    if name == "g3_irr":
        from tests.util import irregular_spd
        rp, cl, vl = irregular_spd(1_585_478, mean_deg=3.83, seed=12345)
        return cga.Matrix(q, vl, cl, rp)
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="p2d_128,p2d_4096,p3d_256,p3d_512,g3_irr")
    ap.add_argument("--mode", type=int, default=0)
    a = ap.parse_args()
    L = lib()
    q = cga.Queue(0)
    for name in a.configs.split(","):
        steps, warm = PLAN[name]
        t0 = time.perf_counter()
        A = matrix(q, name)
        n, nnz = A.N(), A.NNZ()
        sched = A.schedule()
        setup_s = time.perf_counter() - t0
        variant = C.c_int()
        check(L.cgx_csr_variant(sched, C.byref(variant)))
        b = cga.DeviceArray(q, n, np.float64)
        x = cga.DeviceArray(q, n, np.float64)
        check(L.cgx_iota(q.handle, F64, b.ptr, n, 0.0))
        x.fill(0.0)
        cg = C.c_void_p()
        check(L.cgx_cg_create(q.handle, sched, C.byref(cg)))
        check(L.cgx_cg_set_mode(cg, a.mode))
        check(L.cgx_cg_config(cg, 32, 1))
        check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, warm + steps + 1))
        tot, stopped = C.c_int64(), C.c_int()
        check(L.cgx_cg_run(cg, warm, C.byref(tot), C.byref(stopped)))
        check(L.cgx_sync(q.handle))
        t = time.perf_counter()
        check(L.cgx_cg_run(cg, steps, C.byref(tot), C.byref(stopped)))
        check(L.cgx_sync(q.handle))
        dt = time.perf_counter() - t
        ran = tot.value - warm
        its = ran / dt
        balg = 12 * nnz + 4 * (n + 1) + 80 * n
        gbs = balg * its / 1e9
        print(json.dumps({"config": name, "n": n, "nnz": nnz, "bodies_timed": ran,
                          "stopped": stopped.value, "it_per_s": round(its, 1),
                          "ms_per_iter": round(1e3 / its, 4), "B_alg_GB": round(balg / 1e9, 4),
                          "GBps": round(gbs, 1), "frac_of_8TBps": round(gbs / PEAK, 4),
                          "spmv_variant": variant.value, "setup_s": round(setup_s, 2)}),
              flush=True)
        L.cgx_cg_destroy(cg)
        del A, b, x


if __name__ == "__main__":
    main()
