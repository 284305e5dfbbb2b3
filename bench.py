#!/usr/bin/env python3
"""Benchmark of the CG hot path (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]

A "step" is one CG iteration (loop body of CG::solve, src/CG.hpp:359-436):
SpMV + p.Ap, r-update + r.r, x/p-update, on synthetic 3-D 7-point Dirichlet
Poisson CSR (fp64 values, int32 indices, b_i = i + 1, x0 = 0).

* N = 1: the 256^3 grid (the metric's headline config) on one GPU.
* N > 1 (launched with torch.distributed.run, one rank per GPU): weak
  scaling — every rank owns a 256^3 z-slab of a 256 x 256 x (256 N) grid;
  halo exchange of p and the two dot all-reduces go over RCCL.

value = algorithmic HBM bytes of one iteration over the whole job
(B_alg = 12 nnz + 4 (N+1) + 80 N) x iterations/s, in GB/s.
Inputs are generated directly in HBM before the timed region.

The timed region replays hipGraphs of the iteration (no per-kernel events:
recording events between kernels costs ~10 us per kernel). Right after it,
the same solver runs `--profile-steps` more iterations with HIP events around
every kernel on the solver stream; rank 0 reports the dominant kernel's
roofline (k_spmv_dot) from those. At N = 1 rank 0 also times a CPU baseline:
the oracle's OpenMP restatement of the reference's iteration
(oracle/cg_oracle.c) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (before libcgx: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import conjugategradient_amd as cga  # noqa: E402
from conjugategradient_amd._native import F64, check, lib  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters (spec)


def b_alg(n: int, nnz: int) -> int:
    """Algorithmic bytes of one fused CG iteration."""
    return 12 * nnz + 4 * (n + 1) + 80 * n


def spmv_dot_bytes(n: int, nnz: int, fused: bool) -> int:
    """Algorithmic bytes of one launch of the dominant kernel.
    k_spmv_dot (3-kernel mode): val 8 + col 4 per entry, rowptr 4 per row,
    p read 8 and Ap written 8 per row.
    k_spmv_fused (fused mode): the same CSR stream, plus per row r, p_old, x
    read (24) and p_new, x, Ap written (24)."""
    return 12 * nnz + 4 * (n + 1) + (48 if fused else 16) * n


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--grid", type=int, default=256,
                    help="n of the n^3 grid per GPU (weak), or of the global grid (--strong)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: one global n^3 grid split into z-slabs over the GPUs "
                         "(e.g. --grid 512, SURVEY §8(e)); default is weak scaling")
    ap.add_argument("--poll", type=int, default=64, help="iterations per host poll")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-budget-s", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=100,
                    help="iterations timed per kernel with HIP events after the timed region "
                         "(0: skip the roofline pass)")
    ap.add_argument("--mode", type=int, choices=[0, 1, 2, 3], default=0,
                    help="iteration structure (cgx_cg_set_mode): 0 auto, 1 three kernels, "
                         "2 fused (single GPU), 3 three kernels with the x update deferred")
    ap.add_argument("--transport", choices=["rccl", "host"], default="rccl",
                    help="N>1 collectives: RCCL (default) or the host-staged test transport "
                         "(lets ranks share one GPU; rehearsal only, numbers meaningless)")
    return ap.parse_args()


def cpu_baseline(n3: int, threads: int, budget_s: float):
    """The oracle's OpenMP restatement of the reference iteration on a sample
    of the same workload (same matrix, same b), timed on host cores."""
    from oracle import oracle as O

    rp, cl, vl = O.poisson(3, n3, n3, n3)
    n, nnz = len(rp) - 1, len(vl)
    b = np.arange(1, n + 1, dtype=np.float64)
    t1, _ = O.cg_fixed_iters_omp(rp, cl, vl, b, 1, threads)  # probe one iteration
    iters = max(1, min(5000, int(budget_s / max(t1, 1e-6))))  # ~budget_s of CPU work
    t, _ = O.cg_fixed_iters_omp(rp, cl, vl, b, iters, threads)
    its = iters / t
    return {
        "value": round(b_alg(n, nnz) * its / 1e9, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n3}^3 7-pt Poisson, {iters} iterations of the reference command "
                  f"sequence (oracle/cg_oracle.c orc_cg_fixed_iters_omp, OpenMP), "
                  f"{its:.3f} it/s, {t:.2f} s",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    L = lib()
    q = cga.Queue(dev)
    n3 = args.grid
    if args.strong:
        if n3 % world:
            raise SystemExit(f"--strong needs the grid ({n3}) divisible by the GPU count ({world})")
        nz_global = n3
        n_local = n3 * n3 * (n3 // world)
    else:
        nz_global = n3 * world
        n_local = n3 * n3 * n3
    row_begin = rank * n_local
    n_global = n_local * world

    # ---- RCCL communicator (N > 1) ---------------------------------------
    if world > 1 and args.transport == "host":
        from conjugategradient_amd.hostcomm import HostTransport
        transport = HostTransport()
        transport.attach(q)
    elif world > 1:
        uid = C.create_string_buffer(128)
        if rank == 0:
            check(L.cgx_nccl_unique_id(uid, 128))
        obj = [bytes(uid.raw) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        check(L.cgx_dist_init(q.handle, rank, world, obj[0], 128))

    # ---- inputs generated in HBM -------------------------------------------
    nnz_local = L.cgx_poisson_nnz(3, n3, n3, nz_global, row_begin, row_begin + n_local)
    nnz_global = L.cgx_poisson_nnz(3, n3, n3, nz_global, 0, n_global)
    rows = cga.DeviceArray(q, n_local + 1, np.int32)
    cols = cga.DeviceArray(q, nnz_local, np.int32)
    vals = cga.DeviceArray(q, nnz_local, np.float64)
    check(L.cgx_poisson_fill(q.handle, F64, 3, n3, n3, nz_global, row_begin,
                             row_begin + n_local, rows.ptr, cols.ptr, vals.ptr))
    b = cga.DeviceArray(q, n_local, np.float64)
    x = cga.DeviceArray(q, n_local, np.float64)
    check(L.cgx_iota(q.handle, F64, b.ptr, n_local, float(row_begin)))
    x.fill(0.0)
    A = C.c_void_p()
    if world > 1:
        check(L.cgx_csr_create_dist(q.handle, n_global, row_begin, n_local, nnz_local, rows.ptr,
                                    cols.ptr, vals.ptr, F64, C.byref(A)))
    else:
        check(L.cgx_csr_create(q.handle, n_local, nnz_local, rows.ptr, cols.ptr, vals.ptr, F64,
                               None, C.byref(A)))
    variant = C.c_int(0)
    check(L.cgx_csr_variant(A, C.byref(variant)))
    cg = C.c_void_p()
    check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
    check(L.cgx_cg_config(cg, args.poll, 0 if args.no_graph else 1))
    check(L.cgx_cg_set_mode(cg, args.mode))
    fused = args.mode == 2
    total = args.warmup + args.steps + args.profile_steps
    check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, total))
    bodies, stopped = C.c_int64(0), C.c_int(0)
    if args.warmup:
        check(L.cgx_cg_run(cg, args.warmup, C.byref(bodies), C.byref(stopped)))

    # ---- timed region --------------------------------------------------------
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    q.wait()
    t0 = time.perf_counter()
    check(L.cgx_cg_run(cg, args.steps, C.byref(bodies), C.byref(stopped)))
    q.wait()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ran = bodies.value - args.warmup
    if ran != args.steps:
        raise RuntimeError(f"ran {ran} iterations, expected {args.steps} (stopped={stopped.value})")
    its = args.steps / elapsed
    value = b_alg(n_global, nnz_global) * its / 1e9

    # ---- per-kernel HIP-event pass (roofline) ---------------------------------
    avg = (C.c_double * 4)()
    calls = (C.c_int64 * 4)()
    roof = None
    if args.profile_steps:
        check(L.cgx_cg_set_kernel_timing(cg, 1))
        check(L.cgx_cg_run(cg, args.profile_steps, C.byref(bodies), C.byref(stopped)))
        check(L.cgx_cg_kernel_times(cg, avg, calls))
        check(L.cgx_cg_set_kernel_timing(cg, 0))
    if calls[1] > 0:
        kb = spmv_dot_bytes(n_local, nnz_local, fused)
        ach = kb / (avg[1] * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": "k_spmv_fused" if fused else "k_spmv_dot", "bytes_per_launch": kb,
                "avg_us": round(avg[1] * 1e3, 2), "launches_timed": int(calls[1]),
                "other_kernels_avg_us": {"k_update_r": round(avg[2] * 1e3, 2)}}
        # the same launch priced at the bytes its storage format streams (the
        # SELL-P / value-code copy is smaller than CSR, so `frac` on CSR bytes
        # can exceed 1)
        sb = C.c_int64(0)
        check(L.cgx_csr_stream_bytes(A, C.byref(sb)))
        fb = sb.value + (kb - (12 * nnz_local + 4 * (n_local + 1)))
        fach = fb / (avg[1] * 1e-3) / 1e9
        roof.update({"format_bytes_per_launch": fb, "format_achieved": round(fach, 1),
                     "format_frac": round(fach / HBM_PEAK_GBS, 4)})
        if not fused:
            roof["other_kernels_avg_us"]["k_update_xp"] = round(avg[3] * 1e3, 2)
        pmc = os.path.join(ROOT, "profiles", "pmc_spmv_dot.json")
        if os.path.exists(pmc):
            try:
                meta = json.load(open(pmc))
                # PMC bytes of this very kernel: same per-GPU grid, variant, mode
                if (meta.get("grid") == n3 and not args.strong
                        and meta.get("spmv_variant") == variant.value
                        and meta.get("kernel") == roof["kernel"]):
                    roof["traffic"] = meta.get("hbm_bytes_per_launch")
                    roof["traffic_source"] = "profiles/pmc_spmv_dot.json"
            except Exception:
                pass

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu and n3 <= 256:
            cpu = cpu_baseline(n3, min(args.cpu_threads, os.cpu_count() or 1), args.cpu_budget_s)
        line = {
            "metric": "CG iterations/sec + achieved HBM GB/s, 256³ 7-pt Poisson fp64, "
                      "1/2/4/8 GPUs",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "iterations_per_s": round(its, 2),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (3-D 7-point Dirichlet Poisson CSR generated in HBM, "
                    "b_i = i + 1, x0 = 0)",
            "config": {"workload": (f"3D 7-pt Poisson {n3}^3 global, {nz_global // world} z-planes "
                                    f"per GPU" if args.strong else
                                    f"3D 7-pt Poisson {n3}^3 per GPU (global {n3}x{n3}x"
                                    f"{nz_global})") + ", CSR fp64/int32 input, SpMV in the "
                                   "per-matrix best format",
                       "rows_global": n_global, "nnz_global": nnz_global,
                       "bytes_per_iteration": b_alg(n_global, nnz_global),
                       "parallelism": f"rows{world}" if world > 1 else "single",
                       "iteration": {0: "3 kernels, x update deferred over 4 bodies (auto)",
                                     1: "3 kernels", 2: "fused (2 kernels)",
                                     3: "3 kernels, x update deferred over 4 bodies"}[args.mode],
                       "spmv_variant": int(variant.value)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    lib().cgx_cg_destroy(cg)
    lib().cgx_csr_destroy(A)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
