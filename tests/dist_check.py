#!/usr/bin/env python3
"""Multi-rank check of libcgx's RCCL path (cgx_dist.cpp), one process per
rank, launched with torch.distributed.run:

  python -m torch.distributed.run --nproc-per-node W --master-addr 127.0.0.1 \
      --master-port P tests/dist_check.py [--grid 32] [--tol 1e-8] [--mode 3]

Rank r drives device (LOCAL_RANK % visible devices), so W ranks can share
one GPU when the communication library allows it. The global 3-D Poisson
matrix is split in contiguous row blocks; every rank generates its own rows
(global column indices) on the device, builds the halo plan
(cgx_csr_create_dist) and solves with cgx_cg_solve. Rank 0 gathers x and
compares with the oracle (single-process CPU restatement). Prints one JSON
line with the verdict.
"""
from __future__ import annotations

import argparse
import hashlib
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import torch.distributed as dist  # noqa: E402

import conjugategradient_amd as cga  # noqa: E402
from conjugategradient_amd._native import F64, check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--nxy", type=int, default=0,
                    help="nx = ny of the global grid (0: --grid); nz stays --grid")
    ap.add_argument("--bodies", type=int, default=-1,
                    help="fixed body count at tol 0, checked against the oracle's OpenMP "
                         "iteration (for large grids); -1: solve to --tol")
    ap.add_argument("--tol", type=float, default=1e-8)
    ap.add_argument("--transport", choices=["rccl", "host", "host-async", "host-peer", "rccl-peer"],
                    default="rccl",
                    help="setup transport, and '-peer': the device peer transport for the "
                         "iteration (cgx_dist_peer_enable; must pass its self-test); "
                         "'host-async': the host exchange on the comm stream, overlapped "
                         "with the interior slices (cgx_dist_host_async)")
    ap.add_argument("--mode", default="0",
                    help="cgx_cg_set_mode (0 auto, 1, 3, 4); a comma list gives rank r the "
                         "r-th entry (mixed modes across ranks)")
    ap.add_argument("--runs", type=int, default=1,
                    help="split the solve into this many cgx_cg_run calls after one "
                         "cgx_cg_begin (each run ends with its end-of-run flush)")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist.init_process_group("gloo")
    L = lib()
    dev = local % max(1, cga.device_count())
    q = cga.Queue(dev)
    if a.transport.startswith("host"):
        from conjugategradient_amd.hostcomm import HostTransport
        transport = HostTransport()
        transport.attach(q, overlap=a.transport == "host-async")
    else:
        uid = C.create_string_buffer(128)
        if rank == 0:
            check(L.cgx_nccl_unique_id(uid, 128))
        obj = [bytes(uid.raw) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        check(L.cgx_dist_init(q.handle, rank, world, obj[0], 128))
    g = a.grid
    gxy = a.nxy or g
    n = gxy * gxy * g
    base, extra = divmod(n, world)
    counts = [base + (r < extra) for r in range(world)]
    begin = sum(counts[:rank])
    nl = counts[rank]
    nnz = L.cgx_poisson_nnz(3, gxy, gxy, g, begin, begin + nl)
    rows = cga.DeviceArray(q, nl + 1, np.int32)
    cols = cga.DeviceArray(q, nnz, np.int32)
    vals = cga.DeviceArray(q, nnz, np.float64)
    check(L.cgx_poisson_fill(q.handle, F64, 3, gxy, gxy, g, begin, begin + nl, rows.ptr,
                             cols.ptr, vals.ptr))
    A = C.c_void_p()
    check(L.cgx_csr_create_dist(q.handle, n, begin, nl, nnz, rows.ptr, cols.ptr, vals.ptr, F64,
                                C.byref(A)))
    peer = C.c_int(0)
    if a.transport.endswith("-peer"):
        check(L.cgx_dist_peer_enable(A, C.byref(peer)))
        if not peer.value:
            raise SystemExit(f"rank {rank}: peer transport unavailable: "
                             f"{L.cgx_last_error().decode()}")
    coloc, onew = C.c_int(0), C.c_int(0)
    if peer.value:
        check(L.cgx_dist_peer_form(A, C.byref(coloc), C.byref(onew)))
    ghosts, nbrs = C.c_int64(), C.c_int()
    check(L.cgx_csr_halo_info(A, C.byref(ghosts), C.byref(nbrs)))
    ni, nb = C.c_int(), C.c_int()
    check(L.cgx_csr_split_info(A, C.byref(ni), C.byref(nb)))
    # the loop SpMV's form: the lean walk over the interior slices (variant
    # bit 33554432) or the slice-list form
    var = C.c_int()
    check(L.cgx_csr_variant(A, C.byref(var)))
    lc, ls, lg, ld, la, lp = C.c_int(), C.c_int64(), C.c_int(), C.c_int(), C.c_int(), C.c_int()
    check(L.cgx_csr_lean_info(A, C.byref(lc), C.byref(ls), C.byref(lg), C.byref(ld), C.byref(la),
                              C.byref(lp)))
    b = cga.DeviceArray(q, nl, np.float64)
    x = cga.DeviceArray(q, nl, np.float64)
    check(L.cgx_iota(q.handle, F64, b.ptr, nl, float(begin)))
    x.fill(0.0)
    cg = C.c_void_p()
    check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
    modes = [int(m) for m in str(a.mode).split(",")]
    check(L.cgx_cg_set_mode(cg, modes[rank % len(modes)]))
    bodies, rxr = C.c_int64(), C.c_double()
    tol = 0.0 if a.bodies >= 0 else a.tol
    if a.runs > 1:
        check(L.cgx_cg_begin(cg, b.ptr, x.ptr, tol, a.bodies))
        per = max(1, (a.bodies if a.bodies >= 0 else 120) // a.runs)
        stopped = C.c_int(0)
        while not stopped.value:
            check(L.cgx_cg_run(cg, per, C.byref(bodies), C.byref(stopped)))
    else:
        check(L.cgx_cg_solve(cg, b.ptr, x.ptr, tol, a.bodies, C.byref(bodies), C.byref(rxr)))
    mode_run = C.c_int()
    check(L.cgx_cg_get_mode(cg, C.byref(mode_run)))
    modes_run = [None] * world
    dist.all_gather_object(modes_run, int(mode_run.value))
    acalls = C.c_int64()
    check(L.cgx_csr_halo_async_calls(A, C.byref(acalls)))
    acc = C.c_double()
    check(L.cgx_accuracy(q.handle, A, b.ptr, x.ptr, C.byref(acc)))
    parts = [None] * world
    dist.all_gather_object(parts, (int(ghosts.value), int(nbrs.value), (ni.value, nb.value),
                                   int(peer.value), int(acalls.value),
                                   (int(var.value), int(ls.value)),
                                   (int(coloc.value), int(onew.value))))
    # x to rank 0 as tensors, padded to the largest block (gloo gathers
    # equal sizes; blocks differ by at most one row)
    mx = max(counts)
    xl = torch.zeros(mx, dtype=torch.float64)
    xl[:nl] = torch.from_numpy(x.download())
    xs = [torch.empty(mx, dtype=torch.float64) for _ in counts] if rank == 0 else None
    if world > 1:
        dist.gather(xl, xs, dst=0)
    else:
        xs = [xl]
    if rank == 0:
        from oracle import oracle as O
        xg = torch.cat([t[:c] for t, c in zip(xs, counts)]).numpy()
        rp, cl, vl = O.poisson(3, gxy, gxy, g)
        bg = np.arange(1, n + 1, dtype=np.float64)
        dd_equal = None
        if a.bodies >= 0:
            _, xr = O.cg_fixed_iters_omp(rp, cl, vl, bg, a.bodies, 16)
            oracle_bodies = a.bodies
            # the engine's dot model (double-length sums, round 6): x bit for
            # bit whatever the split, where every all-reduce keeps the pairs
            xdd, _ = O.cg_solve_dd(rp, cl, vl, bg, 0.0, threads=16, max_iter=a.bodies)
            dd_equal = bool(np.array_equal(xg, xdd))
        else:
            xr, res = O.cg_solve(rp, cl, vl, bg, a.tol)
            oracle_bodies = res.iterations
        relerr = float(np.linalg.norm(xg - xr) / np.linalg.norm(xr))
        ok = bool(relerr <= 1e-10 and abs(bodies.value - oracle_bodies) <= 2
                  and np.isfinite(xg).all())
        print(json.dumps({"world": world, "transport": a.transport, "mode": a.mode,
                          "mode_run": mode_run.value, "modes_run": modes_run, "runs": a.runs,
                          "grid": [gxy, gxy, g], "bodies": bodies.value,
                          "oracle_bodies": oracle_bodies, "rel_err": relerr,
                          "accuracy": acc.value, "ghosts": [p[0] for p in parts],
                          "neighbours": [p[1] for p in parts],
                          "split": [p[2] for p in parts], "peer": [p[3] for p in parts],
                          "async_exchanges": [p[4] for p in parts],
                          "variant_lean_slices": [p[5] for p in parts],
                          "peer_form": [p[6] for p in parts],
                          "x_sha": hashlib.sha256(xg.tobytes()).hexdigest()[:16],
                          "dd_equal": dd_equal,
                          "ok": ok}), flush=True)
    L.cgx_cg_destroy(cg)
    L.cgx_csr_destroy(A)
    q.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
