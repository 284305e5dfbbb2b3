#!/usr/bin/env python3
"""The partitioned body timed per rank on one GPU (host setup transport,
device peer transport for the iteration: the one-GPU rehearsal of the 8-GPU
path). Every rank owns an nx x ny x planes slab of an nx x ny x (planes W)
grid; for each mode the same bodies run graph-replayed, then a profile pass
times every launch with the events its dispatch records (per-rank kernel
time per body). The ranks share the GPU, so their kernels overlap and each
rank's times include the other ranks' contention: compare modes, not ranks.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tools/dist_rehearsal.py [--nxy 256] [--planes 32] \
        [--modes 3,4] [--steps 400]
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
import torch  # noqa: E402,F401
import torch.distributed as dist  # noqa: E402

import conjugategradient_amd as cga  # noqa: E402
from conjugategradient_amd._native import F64, check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nxy", type=int, default=256)
    ap.add_argument("--planes", type=int, default=32)
    ap.add_argument("--modes", default="3,4")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--profile", type=int, default=100)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist.init_process_group("gloo")
    L = lib()
    q = cga.Queue(0)
    from conjugategradient_amd.hostcomm import HostTransport
    transport = HostTransport()
    transport.attach(q, overlap=False)
    nxy, nz = a.nxy, a.planes * world
    n = nxy * nxy * nz
    nl = n // world
    begin = rank * nl
    nnz = L.cgx_poisson_nnz(3, nxy, nxy, nz, begin, begin + nl)
    rows = cga.DeviceArray(q, nl + 1, np.int32)
    cols = cga.DeviceArray(q, nnz, np.int32)
    vals = cga.DeviceArray(q, nnz, np.float64)
    check(L.cgx_poisson_fill(q.handle, F64, 3, nxy, nxy, nz, begin, begin + nl, rows.ptr,
                             cols.ptr, vals.ptr))
    A = C.c_void_p()
    check(L.cgx_csr_create_dist(q.handle, n, begin, nl, nnz, rows.ptr, cols.ptr, vals.ptr, F64,
                                C.byref(A)))
    ok = C.c_int(0)
    check(L.cgx_dist_peer_enable(A, C.byref(ok)))
    if not ok.value:
        raise SystemExit(f"rank {rank}: peer transport unavailable: {L.cgx_last_error().decode()}")
    var = C.c_int()
    check(L.cgx_csr_variant(A, C.byref(var)))
    b = cga.DeviceArray(q, nl, np.float64)
    check(L.cgx_iota(q.handle, F64, b.ptr, nl, float(begin)))
    from bench import autotune_record
    out = {"world": world, "slab": [nxy, nxy, a.planes], "variant": var.value,
           "forced": os.environ.get("CGX_SPMV_VARIANT"), "autotune": autotune_record(L, A),
           "modes": {}}
    for mode in [int(m) for m in a.modes.split(",")]:
        x = cga.DeviceArray(q, nl, np.float64)
        x.fill(0.0)
        cg = C.c_void_p()
        check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
        check(L.cgx_cg_config(cg, 64, 1))
        # every rank runs the mode or none does (the autotune may give the
        # ranks different forms, and mode 4 needs the lean interior)
        rc = L.cgx_cg_set_mode(cg, mode)
        errs = [None] * world
        dist.all_gather_object(errs, L.cgx_last_error().decode() if rc else None)
        if any(errs):
            out["modes"][str(mode)] = {"error": [e for e in errs]}
            L.cgx_cg_destroy(cg)
            continue
        total = a.warmup + a.steps + a.profile
        check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, total + 1))
        bodies, stopped = C.c_int64(), C.c_int()
        check(L.cgx_cg_run(cg, a.warmup, C.byref(bodies), C.byref(stopped)))
        check(L.cgx_cg_prepare(cg, a.steps))
        q.wait()
        dist.barrier()
        t0 = time.perf_counter()
        check(L.cgx_cg_run(cg, a.steps, C.byref(bodies), C.byref(stopped)))
        q.wait()
        el = time.perf_counter() - t0
        dist.barrier()
        check(L.cgx_cg_set_kernel_timing(cg, 1))
        check(L.cgx_cg_run(cg, a.profile, C.byref(bodies), C.byref(stopped)))
        avg, calls = (C.c_double * 4)(), (C.c_int64 * 4)()
        avgd, callsd = (C.c_double * 4)(), (C.c_int64 * 4)()
        check(L.cgx_cg_kernel_exec_times(cg, avg, calls))
        check(L.cgx_cg_kernel_times(cg, avgd, callsd))
        check(L.cgx_cg_set_kernel_timing(cg, 0))
        # kid 1: the SpMV launches (mode 4: kernels 1 and 2), 2: update_r,
        # 3: the p update (mode 3); exec = the first launch of each kid's
        # dispatch-recorded pair, with_dispatch = the events around all of them
        per = {"ms_per_body": el / a.steps * 1e3,
               "exec_us": [round(avg[i] * 1e3, 2) for i in (1, 2, 3)],
               "with_dispatch_us": [round(avgd[i] * 1e3, 2) for i in (1, 2, 3)],
               "bodies": int(bodies.value)}
        parts = [None] * world
        dist.all_gather_object(parts, per)
        if rank == 0:
            out["modes"][str(mode)] = {
                "us_per_body_max_over_ranks": round(max(p["ms_per_body"] for p in parts) * 1e3,
                                                    2),
                "per_rank": parts}
        L.cgx_cg_destroy(cg)
    if rank == 0:
        print(json.dumps(out), flush=True)
    L.cgx_csr_destroy(A)
    q.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
