"""Where a short timed run loses time (the driver's --steps 20 line runs below
the steady rate of a 400-body run): times repeated cgx_cg_run calls of the
same length on the headline matrix, each from the same slot (so each replays
the same cached graph), after an idle gap or back to back.

  python tools/run20_probe.py [--workload p3d_256] [--steps 20]
"""
import argparse
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="p3d_256")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401

    import conjugategradient_amd as cga
    from conjugategradient_amd import workloads
    from conjugategradient_amd._native import F64, check, lib

    L = lib()
    q = cga.Queue(0)
    wl = workloads.build(L, q, args.workload)
    n = wl.n_local
    b = cga.DeviceArray(q, n, np.float64)
    x = cga.DeviceArray(q, n, np.float64)
    check(L.cgx_iota(q.handle, F64, b.ptr, n, 1.0))
    x.fill(0.0)
    A = C.c_void_p()
    check(L.cgx_csr_create(q.handle, n, wl.nnz_local, wl.rows.ptr, wl.cols.ptr, wl.vals.ptr,
                           F64, None, C.byref(A)))
    cg = C.c_void_p()
    check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
    check(L.cgx_cg_config(cg, 64, 1))
    total = args.warmup + args.steps * (args.reps + 2) + 400
    check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, total))
    bodies, stopped = C.c_int64(0), C.c_int(0)
    check(L.cgx_cg_run(cg, args.warmup, C.byref(bodies), C.byref(stopped)))
    check(L.cgx_cg_prepare(cg, args.steps))
    q.wait()

    def timed(k):
        q.wait()
        t0 = time.perf_counter()
        check(L.cgx_cg_run(cg, k, C.byref(bodies), C.byref(stopped)))
        q.wait()
        return time.perf_counter() - t0

    # the steps are a multiple of 4 bodies: every run starts from the same slot
    for rep in range(args.reps):
        if rep % 2 == 0:
            time.sleep(0.05)  # idle gap, as between cgx_cg_prepare and the timer
        t = timed(args.steps)
        print(f"rep {rep} ({'after 50 ms idle' if rep % 2 == 0 else 'back to back'}): "
              f"{t * 1e3:.3f} ms = {args.steps / t:.1f} it/s", flush=True)
    check(L.cgx_cg_prepare(cg, 400))
    t = timed(400)
    print(f"400 bodies: {t * 1e3:.3f} ms = {400 / t:.1f} it/s "
          f"({t / 400 * 1e6:.1f} us per body)", flush=True)
    check(L.cgx_cg_destroy(cg))
    check(L.cgx_csr_destroy(A))


if __name__ == "__main__":
    main()
