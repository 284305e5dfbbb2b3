#!/usr/bin/env python3
"""One GPU running the per-rank slab of the strong-scaling configs on its
own: 256 x 256 x 32 (256^3 over 8 GPUs) and 512 x 512 x 64 (512^3 over 8),
the same iteration as bench.py (auto mode, graph replay), no halo and no
all-reduce. Its time per body is the floor of an 8-GPU body: the work each
GPU does plus the launch boundaries, without the transport.

    python tools/slab_bench.py [--mode M] [dim,nx,ny,nz,bodies ...]   (M 0: auto)
"""
from __future__ import annotations

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
    L = lib()
    q = cga.Queue(0)
    shapes = ((3, 256, 256, 32, 2000), (3, 512, 512, 64, 400))
    args = sys.argv[1:]
    want_mode = 0
    if len(args) >= 2 and args[0] == "--mode":
        want_mode = int(args[1])
        args = args[2:]
    if args:  # e.g. 2,4096,4096,1,400
        shapes = tuple(tuple(int(v) for v in a.split(",")) for a in args)
    for dim, nx, ny, nz, steps in shapes:
        A = cga.Matrix.poisson(q, dim, nx, ny, nz)
        n = A.N()
        sched = A.schedule()
        team = os.environ.get("CGX_BENCH_TEAM")  # A/B: force the lean walk's team form on / off
        if team is not None and hasattr(L, "cgx_csr_set_lean_team"):
            L.cgx_csr_set_lean_team(sched, int(team))
        b = cga.DeviceArray(q, n, np.float64)
        x = cga.DeviceArray(q, n, np.float64)
        check(L.cgx_iota(q.handle, F64, b.ptr, n, 0.0))
        x.fill(0.0)
        cg = C.c_void_p()
        check(L.cgx_cg_create(q.handle, sched, C.byref(cg)))
        check(L.cgx_cg_config(cg, 64, 1))
        check(L.cgx_cg_set_mode(cg, want_mode))
        mode, v = C.c_int(), C.c_int()
        check(L.cgx_cg_get_mode(cg, C.byref(mode)))
        check(L.cgx_csr_variant(sched, C.byref(v)))
        check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, 20 + steps + 1))
        tot, st = C.c_int64(), C.c_int()
        check(L.cgx_cg_run(cg, 20, C.byref(tot), C.byref(st)))
        check(L.cgx_sync(q.handle))
        t = time.perf_counter()
        check(L.cgx_cg_run(cg, steps, C.byref(tot), C.byref(st)))
        check(L.cgx_sync(q.handle))
        dt = time.perf_counter() - t
        # per-kernel HIP-event pass (eager launches)
        avg = (C.c_double * 4)()
        calls = (C.c_int64 * 4)()
        check(L.cgx_cg_set_kernel_timing(cg, 1))
        check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, 101))
        check(L.cgx_cg_run(cg, 100, C.byref(tot), C.byref(st)))
        # the kernels' own durations (events their dispatches record)
        check(L.cgx_cg_kernel_exec_times(cg, avg, calls))
        print(json.dumps({"slab": [nx, ny, nz], "dim": dim, "rows": n, "mode": mode.value,
                          "spmv_variant": v.value, "bodies": steps,
                          "team": os.environ.get("CGX_BENCH_TEAM"),
                          "us_per_body": round(dt / steps * 1e6, 2),
                          "it_per_s": round(steps / dt, 1),
                          "kernel_us": {"spmv": round(avg[1] * 1e3, 2),
                                        "update_r": round(avg[2] * 1e3, 2),
                                        "p_update_or_flush": round(avg[3] * 1e3, 2)}}),
              flush=True)
        L.cgx_cg_destroy(cg)
        del A, b, x


if __name__ == "__main__":
    main()
