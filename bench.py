#!/usr/bin/env python3
"""Benchmark of the CG hot path (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 256] [--weak]

A "step" is one CG iteration (loop body of CG::solve, src/CG.hpp:359-436):
SpMV + p.Ap, r-update + r.r, x/p-update, on synthetic 3-D 7-point Dirichlet
Poisson CSR (fp64 values, int32 indices, b_i = i + 1, x0 = 0).

* N = 1: the 256^3 grid (the metric's headline config) on one GPU.
* N > 1: strong scaling by default — the same global grid (256^3; --grid 512
  is BASELINE config 4) split into contiguous z-slabs, one rank per GPU;
  the halo exchange of p and the two dot all-reduces run over xGMI: the
  device peer transport when it first solved a small slab problem on this
  node to the RCCL transport's answer (validate_peer: accuracy, body count,
  x to 1e-10; reported as config.transport_validation), else RCCL. --weak
  gives every rank its own 256^3 slab instead.
* `python bench.py --gpus N` with no launcher environment starts its own N
  ranks (torch.distributed.run, 127.0.0.1) as a child process before touching
  any GPU; under a launcher, WORLD_SIZE must equal --gpus.

value = CG iterations (bodies) per second of the whole job, the metric's first
quantity (round 6: it was the GB/s figure below, which a body that moves
fewer bytes — mode 6, Ap formed again instead of stored — lowers while it
raises iterations/s). achieved_GBs = the COMPULSORY HBM bytes of one
iteration in the formats the kernels stream (the SpMV's matrix stream from
cgx_csr_stream_bytes, p read and Ap written — mode 6: p read twice, no Ap —,
24 N for the r update, 34 N average for the deferred x/p update), summed
over ranks, x iterations/s, in GB/s: a physical figure (<= peak), and
iteration_frac = achieved_GBs / (peak x N). The CSR-priced figure of SURVEY
§8(d) (B_alg = 12 nnz + 4 (N+1) + 80 N) is reported beside it as
`csr_equivalent_GBs`.

The timed region replays hipGraphs of the iteration (no per-kernel events).
Right after it, `--profile-steps` more iterations run with HIP events around
every kernel on the solver stream (the stream the kernels run on); rank 0
reports the dominant kernel's roofline (k_spmv_dot) from those, priced at
its own format's compulsory bytes. At N = 1 rank 0 also reports:
  * `csr_general`: the same 256^3 matrix solved with the general-value
    formats (plain SELL-P values, and CSR-stream — the path of a matrix with
    many distinct values such as G3_circuit);
  * `cpu_baseline`: the oracle's OpenMP restatement of the reference
    iteration (oracle/cg_oracle.c) on every core this job may use, on a
    bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters (spec)
KVL = 33554432  # variant bit of the lean stencil walk (include/cgx.h cgx_csr_lean_info)
METRIC = "CG iterations/sec + achieved HBM GB/s, 256³ 7-pt Poisson fp64, 1/2/4/8 GPUs"


def b_alg(n: int, nnz: int) -> int:
    """CSR-priced bytes of one fused CG iteration."""
    return 12 * nnz + 4 * (n + 1) + 80 * n


def csr_spmv_bytes(n: int, nnz: int) -> int:
    """CSR-priced bytes of one k_spmv_dot launch: val 8 + col 4 per entry,
    rowptr 4 per row, p read 8 and Ap written 8 per row."""
    return 12 * nnz + 4 * (n + 1) + 16 * n


def update_bytes_per_iter(n: int, mode: int) -> int:
    """Compulsory bytes of the two vector kernels of one body.
    k_update_r: r, Ap read, r written (24 n). The x/p update: mode 1 reads x,
    p, r and writes x, p (40 n); mode 3 (default) writes p_{k+1} from r, p_k
    (24 n) in three bodies of four and in the fourth also applies
    x += a0 p0 + .. + a3 p3 (reads x and the three other p buffers, writes x:
    +40 n), 34 n on average."""
    if mode in (4, 7):  # the p update is folded into the SpMV (spmv_bytes_per_iter);
        # the slot-3 x flush: x r/w + 4 p reads, once per 4 bodies (mode 7:
        # kernel 2 reads p_k where update_r reads Ap, plus its matrix stream)
        return 24 * n + 12 * n
    # mode 6: kernel 2 reads p (A p formed again) where update_r reads Ap: the
    # same 24 n, plus its matrix stream (added by the caller)
    xp = 40 * n if mode in (1, 5) else 34 * n  # mode 5: priced as mode 1
    return 24 * n + xp


def spmv_bytes_per_iter(stream_bytes: int, n: int, mode: int) -> int:
    """The SpMV launch: its matrix stream (cgx_csr_stream_bytes) + p read + Ap
    written (16 n); mode 4's k_spmv_fd reads r and p_{k-1} and writes p_k and
    Ap (32 n)."""
    return stream_bytes + (32 * n if mode == 4 else 8 * n if mode == 6 else
                           24 * n if mode == 7 else 16 * n)


def warmup_run(args) -> int:
    """Untimed bodies before the window: --warmup rounded up to whole slot
    cycles (4). The iteration rotates p over 4 slots and applies the deferred
    x update of a group of 4 bodies in its slot-3 launch, so a window that
    starts at slot 0 and holds whole groups carries every body's x update and
    no partial-group flush (which a window starting at slot 1 pays once at its
    end while the first group's x update fell in the warm-up: +2.3% at
    256^3 over 20 steps, profiles/r6p_*). The line reports both counts."""
    return args.warmup if args.legacy_window else -(-args.warmup // 4) * 4


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="p3d_256",
                    choices=["p3d_256", "p3d_512", "p2d_4096", "p2d_128", "g3_standin"],
                    help="BASELINE.json configuration (conjugategradient_amd/workloads.py); "
                         "the default is the headline 256^3 one; N > 1 takes the 3-D ones")
    ap.add_argument("--grid", type=int, default=None,
                    help="n of the global n^3 grid of a 3-D workload (strong scaling, the "
                         "default), or of each rank's slab with --weak; --grid 512 is p3d_512")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: every rank owns an n^3 slab of an n x n x (n N) grid")
    ap.add_argument("--strong", action="store_true", help=argparse.SUPPRESS)  # the default
    ap.add_argument("--poll", type=int, default=64, help="iterations per host poll")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: every core this job may use)")
    ap.add_argument("--cpu-budget-s", type=float, default=40.0,
                    help="wall-clock budget of the CPU baseline's runs (SURVEY §8(d): 5 runs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-general", action="store_true",
                    help="skip the csr_general block (general-value formats)")
    ap.add_argument("--profile-steps", type=int, default=100,
                    help="iterations timed per kernel with HIP events after the timed region "
                         "(0: skip the roofline pass)")
    ap.add_argument("--mode", type=int, choices=[0, 1, 2, 3, 4, 5, 6, 7], default=0,
                    help="iteration structure (cgx_cg_set_mode): 0 auto, 1 three kernels, "
                         "2 fused (single GPU), 3 three kernels with the x update deferred, "
                         "4 two kernels (p update folded into the SpMV), x deferred")
    ap.add_argument("--transport", choices=["auto", "rccl", "peer", "host", "host-peer"],
                    default="auto",
                    help="N>1 collectives: auto (device peer transport over xGMI when it "
                         "solves a validation problem to RCCL's answer on this node, else "
                         "RCCL), rccl, peer (fail if unavailable), "
                         "host (host-staged test transport: lets ranks share one GPU; "
                         "rehearsal only, numbers meaningless), host-peer (host setup, "
                         "device peer iteration: a one-GPU rehearsal of the peer path)")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 PMC passes that measure roofline.traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--lean-team", choices=["auto", "0", "1"], default="auto",
                    help=argparse.SUPPRESS)  # A/B: the lean walk's team form off / on
    ap.add_argument("--master-port", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--force-lean", action="store_true", help=argparse.SUPPRESS)
    # A/B: --warmup bodies exactly, the graphs captured after them
    ap.add_argument("--legacy-window", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher: `bench.py --gpus N` outside torch.distributed.run
# ---------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher_cmd(args, argv) -> list[str]:
    """The torch.distributed.run command line that starts args.gpus ranks of
    this script with the same arguments (rendezvous on 127.0.0.1)."""
    port = args.master_port or _free_port()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
            f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def maybe_launch(args, argv) -> int | None:
    """Start the ranks as a child process when --gpus N > 1 and no launcher
    environment exists (nothing has touched a GPU yet: the parent never
    initialises HIP). Returns the child's exit code, or None to run here."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus <= 1:
            return None
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        return subprocess.call(launcher_cmd(args, argv), env=env)
    if int(world) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: they must match")
    return None


# ---------------------------------------------------------------------------
# CPU baseline
# ---------------------------------------------------------------------------
def job_cores() -> dict:
    """Cores this job may run on: the affinity mask, capped by a cgroup CPU
    quota and by the job's declared CPU share (OMP_NUM_THREADS) when set;
    plus nproc and the CPU model for the record."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except Exception:
        pass
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    use = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    # the GPU box declares this job's CPU share in OMP_NUM_THREADS (16 per
    # GPU; nproc there counts the whole machine): stay within it
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        use = min(use, int(share))
    return {"use": int(use), "affinity": int(aff), "cgroup_quota": quota,
            "declared_share": int(share) if share and share.isdigit() else None,
            "nproc": os.cpu_count(), "model": model}


def cpu_baseline(workload: str, grid, threads: int, budget_s: float, iters: int = 500,
                 warmup: int = 20, reps: int = 5):
    """The oracle's OpenMP restatement of the reference iteration on the same
    workload (same matrix, same b), timed on host cores to the SURVEY §8(d)
    protocol: `iters` (500) timed bodies after `warmup` (20) untimed ones,
    the median of `reps` (5) runs, or of as many runs as fit in `budget_s`
    (at least one; the sample names the count)."""
    import numpy as np
    from oracle import oracle as O

    from conjugategradient_amd import workloads

    info = job_cores()
    if threads <= 0:
        threads = info["use"]
    if workload in workloads.POISSON:
        dim, nx, ny, nz = workloads.POISSON[workload]
        if grid and dim == 3:
            nx = ny = nz = grid
        rp, cl, vl = O.poisson(dim, nx, ny, nz)
        what = f"{nx}^3 7-pt Poisson" if dim == 3 else f"{nx}^2 5-pt Poisson"
    else:
        rp, cl, vl = workloads.host_csr(workload)
        what = workload
    n, nnz = len(rp) - 1, len(vl)
    b = np.arange(1, n + 1, dtype=np.float64)
    times = []
    t_start = time.perf_counter()
    while len(times) < reps:
        t, _ = O.cg_timed_omp(rp, cl, vl, b, warmup, iters, threads)
        times.append(t)
        spent = time.perf_counter() - t_start
        if spent + spent / len(times) > budget_s:  # the next run would pass the budget
            break
    med = float(np.median(times))
    its = iters / med
    return {
        "value": round(its, 3),  # the line's unit (value is iterations/s from round 6)
        "unit": "it/s",
        "cores": threads,
        "kind": "port",
        "iterations_per_s": round(its, 3),
        "csr_equivalent_GBs": round(b_alg(n, nnz) * its / 1e9, 3),
        "protocol": {"timed_iterations": iters, "warmup_iterations": warmup,
                     "runs": len(times), "runs_asked": reps, "statistic": "median",
                     "run_seconds": [round(x, 3) for x in times]},
        "host": {"cpu_model": info["model"], "nproc": info["nproc"],
                 "affinity_cores": info["affinity"], "cgroup_cpu_quota": info["cgroup_quota"],
                 "declared_cpu_share": info["declared_share"],
                 "omp_proc_bind": os.environ.get("OMP_PROC_BIND")},
        "sample": f"{what}: K = {iters} timed iterations of the reference command sequence "
                  f"after {warmup} untimed warm-up iterations (oracle/cg_oracle.c "
                  f"orc_cg_timed_omp, OpenMP, {threads} threads), median of {len(times)} "
                  f"run(s) of {reps} asked within a {budget_s:.0f} s budget: {its:.3f} it/s "
                  f"(csr_equivalent_GBs: priced at the CSR bytes B_alg)",
    }


TUNE_KINDS = {0: "k_spmv_dot", 1: "k_spmv_dot (interior slices)", 2: "k_spmv_fd",
              3: "lean walk", 4: "lean walk (interior slices)",
              5: "k_spmv_fd lean walk, team form",
              6: "the pick so far, re-timed beside the lean walk",
              7: "boundary rows (CSR-stream launch; added to the interior forms)"}


SETUP_PHASES = ("schedule", "sell_plan_pack", "value_codes", "split", "autotune", "rest")


def setup_record(L, A, wall_s: float) -> dict:
    """cgx_csr_create's cost (the matrix's setup, outside the timed region):
    the wall time of the call and its phases (cgx_csr_setup_times)."""
    from conjugategradient_amd._native import check

    rec = {"csr_create_s": round(wall_s, 4)}
    if hasattr(L, "cgx_csr_setup_times"):
        ms, n = (C.c_double * 6)(), C.c_int(0)
        check(L.cgx_csr_setup_times(A, ms, 6, C.byref(n)))
        rec["phases_ms"] = {SETUP_PHASES[k]: round(ms[k], 1) for k in range(min(6, n.value))}
    return rec


def autotune_record(L, A) -> dict | None:
    """The SpMV autotune's timings of this matrix (cgx_csr_autotune_record):
    every form it timed, how, and its median µs per launch."""
    n = C.c_int(0)
    if not hasattr(L, "cgx_csr_autotune_record"):  # (an older A/B build, tools/ab_lib.py)
        return None
    L.cgx_csr_autotune_record(A, None, None, None, 0, C.byref(n))
    if n.value == 0:
        return None
    v, k, us = (C.c_int * n.value)(), (C.c_int * n.value)(), (C.c_float * n.value)()
    L.cgx_csr_autotune_record(A, v, k, us, n.value, C.byref(n))
    return {"rule": "median of 5 interleaved rounds of 3 launches per form; a form displaces "
                    "the more specialised one only when >= 3% faster (a split matrix: its "
                    "interior forms' times plus the boundary rows' launch)",
            "forms": [{"variant": int(v[i]), "how": TUNE_KINDS.get(k[i], str(k[i])),
                       "us": round(float(us[i]), 2)} for i in range(n.value)]}


def rccl_timing(L, q, args, wl, b, x, transport, its, elapsed, world, dist) -> dict:
    """The same bodies over RCCL (ncclSend/Recv halo on the comm stream
    beside the interior slices, ncclAllReduce for p.Ap and r.r; SURVEY
    §8(e), the north star's transport) when the timed run used the device
    peer transport: a second partitioned matrix without the peer transport,
    the same warmup and steps, max over ranks. `skipped` says why not."""
    import torch

    from conjugategradient_amd._native import F64, check

    if transport == "rccl":
        return {"iterations_per_s": round(its, 2), "ms_per_step": round(elapsed / args.steps * 1e3,
                                                                         4),
                "note": "the timed run itself (RCCL carried it)"}
    if not transport.startswith("peer (setup: rccl"):
        return {"skipped": f"no RCCL communicator (setup transport {transport!r}: RCCL refuses "
                           "ranks that share one GPU, so the one-GPU rehearsal runs the host "
                           "transport)"}
    A2 = C.c_void_p()
    check(L.cgx_csr_create_dist(q.handle, wl.n_global, wl.row_begin, wl.n_local, wl.nnz_local,
                                wl.rows.ptr, wl.cols.ptr, wl.vals.ptr, F64, C.byref(A2)))
    cg = C.c_void_p()
    check(L.cgx_cg_create(q.handle, A2, C.byref(cg)))
    check(L.cgx_cg_config(cg, args.poll, 0 if args.no_graph else 1))
    # (partitioned mode 4 needs the device peer transport: RCCL runs mode 3)
    check(L.cgx_cg_set_mode(cg, 3 if args.mode == 4 else args.mode))
    # its own x: the timed run's cg continues in the profile pass after this
    # (modes 3 / 4 hold deferred x updates for its x)
    import numpy as np

    import conjugategradient_amd as cga
    x2 = cga.DeviceArray(q, wl.n_local, np.float64)
    x2.fill(0.0)
    warm = warmup_run(args)
    check(L.cgx_cg_begin(cg, b.ptr, x2.ptr, 0.0, warm + args.steps))
    bodies, stopped = C.c_int64(0), C.c_int(0)
    if warm:
        check(L.cgx_cg_run(cg, warm, C.byref(bodies), C.byref(stopped)))
    check(L.cgx_cg_prepare(cg, args.steps))
    q.wait()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    check(L.cgx_cg_run(cg, args.steps, C.byref(bodies), C.byref(stopped)))
    q.wait()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    el = t1 - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ok = bodies.value - warm == args.steps
    check(L.cgx_cg_destroy(cg))
    check(L.cgx_csr_destroy(A2))
    if not ok:
        return {"skipped": f"the RCCL run stopped early (stopped={stopped.value})"}
    return {"iterations_per_s": round(args.steps / el, 2),
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "note": "the same workload and bodies over RCCL (halo: ncclSend/Recv on the comm "
                    "stream; dots: ncclAllReduce), no device peer transport"}


# ---------------------------------------------------------------------------
# the measured run (one rank)
# ---------------------------------------------------------------------------
def run(args) -> None:
    import numpy as np
    import torch  # noqa: F401  (before libcgx: one HIP runtime per process)
    import torch.distributed as dist

    import conjugategradient_amd as cga
    from conjugategradient_amd import workloads
    from conjugategradient_amd._native import F64, check, lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    dev = local % max(1, cga.device_count())
    L = lib()
    q = cga.Queue(dev)
    strong = not args.weak
    # ---- communicator (N > 1) ----------------------------------------------
    transport = "single"
    rccl_note = None
    # the distributed path: N > 1, or --transport rccl at N = 1 (the RCCL
    # iteration on one rank: all-reduces over a one-rank communicator)
    dist_on = world > 1 or args.transport == "rccl"
    if world > 1 and args.transport in ("host", "host-peer"):
        from conjugategradient_amd.hostcomm import HostTransport
        ht = HostTransport()
        ht.attach(q)
        transport = "host"
    elif dist_on:
        # RCCL; with --transport auto, a node where it does not come up
        # (every rank's outcome, agreed over gloo) keeps the host transport
        # for setup and tries the device peer transport for the iteration
        uid = C.create_string_buffer(128)
        rc = 0
        if rank == 0:
            rc = L.cgx_nccl_unique_id(uid, 128)
        obj = [(bytes(uid.raw), rc) if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(obj, src=0)
        if obj[0][1] == 0:
            rc = L.cgx_dist_init(q.handle, rank, world, obj[0][0], 128)
        else:
            rc = obj[0][1]
        why = L.cgx_last_error().decode() if rc else ""
        ok = torch.tensor([0.0 if rc == 0 else 1.0], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(ok)
        if ok.item() == 0.0:
            transport = "rccl"
        elif args.transport == "auto":
            if rc == 0:  # this rank's communicator came up alone: a fresh context
                q = cga.Queue(dev)
            from conjugategradient_amd.hostcomm import HostTransport
            ht = HostTransport()
            ht.attach(q)
            transport = "host"
            rccl_note = f"RCCL unavailable ({why or 'on another rank'}): host setup transport"
        else:
            raise SystemExit(f"bench.py: RCCL init failed: {why or 'on another rank'}")
    wr, ww = C.c_int(0), C.c_int(0)
    check(L.cgx_dist_rank(q.handle, C.byref(wr), C.byref(ww)))
    if ww.value != args.gpus or ww.value != world:
        raise SystemExit(f"bench.py: communicator world {ww.value}, --gpus {args.gpus}, "
                         f"WORLD_SIZE {world}: they must match")

    # ---- inputs in HBM (conjugategradient_amd/workloads.py) -------------------
    wl = workloads.build(L, q, args.workload, world, rank, args.grid, args.weak)
    n_local, nnz_local, n_global, nnz_global = wl.n_local, wl.nnz_local, wl.n_global, \
        wl.nnz_global
    row_begin = wl.row_begin
    b = cga.DeviceArray(q, n_local, np.float64)
    x = cga.DeviceArray(q, n_local, np.float64)
    check(L.cgx_iota(q.handle, F64, b.ptr, n_local, float(row_begin)))
    x.fill(0.0)
    A = C.c_void_p()
    q.wait()
    t_setup = time.perf_counter()
    if dist_on:
        check(L.cgx_csr_create_dist(q.handle, n_global, row_begin, n_local, nnz_local,
                                    wl.rows.ptr, wl.cols.ptr, wl.vals.ptr, F64, C.byref(A)))
    else:
        check(L.cgx_csr_create(q.handle, n_local, nnz_local, wl.rows.ptr, wl.cols.ptr,
                               wl.vals.ptr, F64, None, C.byref(A)))
    q.wait()
    setup = setup_record(L, A, time.perf_counter() - t_setup)
    if args.lean_team != "auto" and not dist_on:  # A/B of the lean walk's team form
        check(L.cgx_csr_set_lean_team(A, int(args.lean_team)))
    if args.force_lean:  # the lean walk whatever the autotune chose (tests)
        check(L.cgx_csr_set_variant(A, KVL))
    peer_note = None
    peer_form = None
    validation = None
    use_peer = world > 1 and args.transport in ("peer", "host-peer")
    if world > 1 and args.transport in ("auto", "host-peer"):
        # the device peer transport is used only after it solved a small slab
        # problem on THIS node to the same answer as the setup transport
        # (validate_peer; RCCL, or the host transport of the one-GPU
        # rehearsal); otherwise the numbers come from the setup transport
        validation = validate_peer(L, q, world, rank, dist)
        use_peer = validation["ok"]
        if not use_peer and args.transport == "host-peer":
            raise SystemExit(f"bench.py: peer transport failed its validation: "
                             f"{validation.get('why')}")
        if not use_peer:
            peer_note = validation.get("why")
    if use_peer:
        # verified by a self-test on every rank; all ranks agree on the
        # outcome (else the setup transport stays)
        ok = C.c_int(0)
        check(L.cgx_dist_peer_enable(A, C.byref(ok)))
        if ok.value:
            transport = "peer (setup: " + transport + ")"
            coloc, onew = C.c_int(0), C.c_int(0)
            check(L.cgx_dist_peer_form(A, C.byref(coloc), C.byref(onew)))
            peer_form = {"colocated": coloc.value, "one_waiter": onew.value}
        elif args.transport != "auto":
            raise SystemExit(f"bench.py: peer transport unavailable: "
                             f"{L.cgx_last_error().decode()}")
        else:
            peer_note = L.cgx_last_error().decode()
    variant = C.c_int(0)
    check(L.cgx_csr_variant(A, C.byref(variant)))
    sbytes = C.c_int64(0)
    check(L.cgx_csr_stream_bytes(A, C.byref(sbytes)))
    ntpl, tpl_slices = C.c_int(0), C.c_int64(0)
    check(L.cgx_csr_templates(A, C.byref(ntpl), C.byref(tpl_slices)))
    lean = [C.c_int(0), C.c_int64(0), C.c_int(0), C.c_int(0), C.c_int(0), C.c_int(0)]
    check(L.cgx_csr_lean_info(A, *[C.byref(v) for v in lean]))
    lean_on = bool(variant.value & KVL)
    team = C.c_int(0)
    if lean_on and hasattr(L, "cgx_csr_lean_team"):
        check(L.cgx_csr_lean_team(A, C.byref(team)))
    sfx = "_t" if team.value else ""  # the walk's team form (1,024-thread workgroups)
    autotune = autotune_record(L, A)
    cg = C.c_void_p()
    check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
    check(L.cgx_cg_config(cg, args.poll, 0 if args.no_graph else 1))
    check(L.cgx_cg_set_mode(cg, args.mode))
    fused = args.mode == 2
    me = C.c_int(0)
    check(L.cgx_cg_get_mode(cg, C.byref(me)))
    if dist_on and world > 1 and args.mode == 0:
        # the ranks agree on the body: each rank's autotune picks its own
        # interior form and auto mode 4 needs the lean one, so mode 4 runs only
        # where every rank took it, and only after it solved a 128 x 128 slab
        # per rank over the peer transport to the setup transport's answer
        import torch
        t4 = torch.tensor([1.0 if me.value == 4 else 0.0], dtype=torch.float64)
        dist.all_reduce(t4, op=dist.ReduceOp.MIN)
        why4 = None if t4.item() == 1.0 else "not every rank's interior takes it"
        if why4 is None:
            v4 = validate_peer(L, q, world, rank, dist, nxy=128, mode=4)
            validation = {**(validation or {}), "mode4": v4}
            if not v4["ok"]:
                why4 = f"failed its validation ({v4.get('why')})"
        if why4 is not None and me.value == 4:
            check(L.cgx_cg_set_mode(cg, 3))
            check(L.cgx_cg_get_mode(cg, C.byref(me)))
            peer_note = (peer_note or "") + f" partitioned mode 4 {why4}: mode 3"
    if dist_on and me.value == 4:
        sfx = "_push"  # partitioned mode 4: the interior walk with the push in front
    mode_eff = me.value
    warm = warmup_run(args)
    total = warm + args.steps + args.profile_steps
    check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, total))
    bodies, stopped = C.c_int64(0), C.c_int(0)
    if args.legacy_window:
        if warm:
            check(L.cgx_cg_run(cg, warm, C.byref(bodies), C.byref(stopped)))
        check(L.cgx_cg_prepare(cg, args.steps))
    else:
        # the graphs the timed run replays are captured first (from slot 0,
        # where the whole-cycle warm-up leaves the slot), so the warm-up bodies
        # run right before the window instead of before the captures
        check(L.cgx_cg_prepare(cg, args.steps))
        if warm:
            check(L.cgx_cg_run(cg, warm, C.byref(bodies), C.byref(stopped)))

    # ---- timed region ----------------------------------------------------------
    # the solver's stream is the only one with work (q.wait() drains it; the
    # run itself returns after its last chunk finished)
    q.wait()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    check(L.cgx_cg_run(cg, args.steps, C.byref(bodies), C.byref(stopped)))
    q.wait()
    t1 = time.perf_counter()
    if args.pmc_child:  # a PMC pass of pmc_traffic: the dispatches are what it needs
        check(L.cgx_cg_destroy(cg))
        check(L.cgx_csr_destroy(A))
        return
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ran = bodies.value - warm
    if ran != args.steps:
        raise RuntimeError(f"ran {ran} iterations, expected {args.steps} (stopped={stopped.value})")
    its = args.steps / elapsed
    # the north star's transport (RCCL halo + all-reduces) timed beside the
    # device peer one when the peer transport carried the run
    rccl_iteration = None
    if dist_on:
        rccl_iteration = rccl_timing(L, q, args, wl, b, x, transport, its, elapsed, world, dist)

    # compulsory bytes of one iteration in the streamed formats, all ranks
    spmv_fmt_local = spmv_bytes_per_iter(sbytes.value, n_local, mode_eff)
    iter_local = spmv_fmt_local + update_bytes_per_iter(n_local, mode_eff)
    if mode_eff in (6, 7):  # kernel 2's walk streams the matrix's format again
        iter_local += sbytes.value
    if fused:
        iter_local = sbytes.value + 48 * n_local + 24 * n_local
    iter_global = iter_local
    if world > 1:
        tb = torch.tensor([float(iter_local)], dtype=torch.float64)
        dist.all_reduce(tb)
        iter_global = int(tb.item())
    value = iter_global * its / 1e9
    csr_eq = b_alg(n_global, nnz_global) * its / 1e9

    # ---- per-kernel HIP-event pass (roofline) ------------------------------------
    avg = (C.c_double * 4)()
    calls = (C.c_int64 * 4)()
    roof = None
    avg_d = (C.c_double * 4)()  # event pairs around each launch (dispatch included)
    if args.profile_steps:
        check(L.cgx_cg_set_kernel_timing(cg, 1))
        check(L.cgx_cg_run(cg, args.profile_steps, C.byref(bodies), C.byref(stopped)))
        check(L.cgx_cg_kernel_times(cg, avg_d, calls))
        # the kernels' own durations: event pairs their dispatches record
        # (hipExtLaunchKernel), as rocprofv3 times them; the launch-bracketing
        # pairs where a kernel does not record them
        xcalls = (C.c_int64 * 4)()
        if hasattr(L, "cgx_cg_kernel_exec_times"):  # (an older A/B build lacks it, tools/ab_lib.py)
            check(L.cgx_cg_kernel_exec_times(cg, avg, xcalls))
        for i in range(4):
            if xcalls[i] == 0:
                avg[i] = avg_d[i]
        check(L.cgx_cg_set_kernel_timing(cg, 0))
    if calls[1] > 0 and mode_eff == 5:
        roof = coop_roofline(L, cg, avg, calls, args.profile_steps, iter_local)
    elif calls[1] > 0:
        kb = spmv_fmt_local + (32 * n_local if fused else 0)
        # mode 6: the walk runs in kernels 1 (p.Ap only) and 2 (r updated in
        # its epilogue); kernel 2 is the larger, and the roofline's
        kid = 2 if mode_eff == 6 else 1
        if mode_eff == 6:
            kb = sbytes.value + 24 * n_local
        if mode_eff == 7:  # two walks of 24 N each: the longer one
            kid = 2 if avg[2] >= avg[1] else 1
            kb = sbytes.value + 24 * n_local
        ach = kb / (avg[kid] * 1e-3) / 1e9
        cb = csr_spmv_bytes(n_local, nnz_local) + (32 * n_local if fused else 0) + \
            (16 * n_local if mode_eff == 4 else 0)
        kname = {2: "k_spmv_fused", 4: "k_spmv_fd_lean" + sfx if lean_on else "k_spmv_fd",
                 6: "k_spmv_lean_updr",
                 7: "k_spmv_lean_updr_rule" if kid == 2 else "k_spmv_fd_dot_tile"
                 }.get(mode_eff, "k_spmv_lean" if lean_on else "k_spmv_dot")
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": kname,
                "bytes_per_launch": kb,
                "bytes_basis": ("compulsory bytes of the kernel's own format: matrix stream "
                                "(cgx_csr_stream_bytes) + p_k read + r read + r written (A "
                                "p_k formed again, no Ap vector)" if kname.startswith(
                                    "k_spmv_lean_updr") else
                                "compulsory bytes of the kernel's own format: matrix stream "
                                "(cgx_csr_stream_bytes) + r read + p_{k-1} read + p_k written "
                                "(no Ap vector)" if kname == "k_spmv_fd_dot_tile" else
                                "compulsory bytes of the kernel's own format: matrix stream "
                                "(cgx_csr_stream_bytes) + p read + Ap written" +
                                (" + r read + p_k written" if mode_eff == 4 else "")),
                "avg_us": round(avg[kid] * 1e3, 2), "launches_timed": int(calls[kid]),
                "avg_us_basis": "HIP events recorded by each launch's dispatch "
                                "(hipExtLaunchKernel start/stop) on the solver stream",
                "avg_us_with_dispatch": round(avg_d[kid] * 1e3, 2),
                "csr_equivalent_bytes_per_launch": cb,
                "csr_equivalent_GBs": round(cb / (avg[kid] * 1e-3) / 1e9, 1),
                "other_kernels_avg_us": {"k_update_r": round(avg[2] * 1e3, 2)}}
        if mode_eff == 4:  # every fourth k_update_r also applies the group's x updates
            roof["other_kernels_avg_us"] = {"k_update_r (+ x flush in 1 of 4)":
                                            round(avg[2] * 1e3, 2)}
        elif mode_eff == 7:
            other = 1 if kid == 2 else 2
            roof["other_kernels_avg_us"] = {
                ("k_spmv_fd_dot_tile" if other == 1 else "k_spmv_lean_updr_rule"):
                    round(avg[other] * 1e3, 2),
                "k_flush_group (slot 3 only)": round(avg[3] * 1e3, 2)}
            roof["other_walk_frac"] = round(kb / (avg[other] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        elif mode_eff == 6:
            kb1 = sbytes.value + 8 * n_local  # the walk's p.Ap: matrix stream + p read
            roof["other_kernels_avg_us"] = {"k_spmv_lean_dot": round(avg[1] * 1e3, 2),
                                            "k_update_p": round(avg[3] * 1e3, 2)}
            roof["k_spmv_lean_dot"] = {"bytes_per_launch": kb1, "avg_us": round(avg[1] * 1e3, 2),
                                       "frac": round(kb1 / (avg[1] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                                     4)}
        elif not fused:
            roof["other_kernels_avg_us"]["k_update_p"] = round(avg[3] * 1e3, 2)
        if world == 1 and not args.no_traffic:
            # HBM bytes per launch from rocprofv3 PMC passes of this same
            # workload, variant and mode (child processes, after this run)
            # (a lean walk is forced at the grid its class layout was built for)
            t = pmc_traffic(args, f"{int(variant.value)}:{lean[2].value}" if lean_on
                            else str(int(variant.value)), mode_eff, team.value)
            roof["traffic_by_kernel"] = t.get("by_kernel")
            roof["traffic_method"] = t.get("method")
            key = ("k_spmv_fd_lean_t<double, true, true>" if kname == "k_spmv_fd_lean_t"
                   else f"{kname}<double>" if kname.startswith(("k_spmv_lean", "k_spmv_fd_lean",
                                                                 "k_spmv_fd_dot"))
                   else f"{kname}<double, {int(variant.value & ~KVL)}>")
            if t.get("by_kernel") and key in t["by_kernel"]:
                roof["traffic"] = t["by_kernel"][key]
                roof["traffic_ratio_to_compulsory"] = round(roof["traffic"] / kb, 4)
            else:
                roof["traffic_error"] = t.get("error") or f"no PMC samples for {key}"

    # ---- general-value formats on the same matrix (N = 1) --------------------------
    general = None
    if world == 1 and rank == 0 and not args.no_general and mode_eff == 5:
        general = {"skipped": "mode 5 (persistent body) reads the CSR arrays directly; the "
                              "SpMV formats do not enter it"}
    elif world == 1 and rank == 0 and not args.no_general:
        general = general_formats(L, q, A, b, x, n_local, nnz_local, mode_eff, args)

    line = None
    if rank == 0:
        cpu = None
        big = args.workload == "p3d_512" or (args.grid or 0) > 256
        if world == 1 and not args.no_cpu and not big:
            os.environ.setdefault("OMP_PROC_BIND", "close")
            cpu = cpu_baseline(args.workload, args.grid, args.cpu_threads, args.cpu_budget_s)
        workload = wl.description
        line = {
            "metric": METRIC,
            "value": round(its, 2),
            "unit": "it/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_run": warm,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "iterations_per_s": round(its, 2),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (Dirichlet Poisson CSR generated in HBM, b_i = i + 1, x0 = 0)"
                     if args.workload in workloads.POISSON else
                     "synthetic (see config.workload; b_i = i + 1, x0 = 0)"),
            "value_basis": "CG iterations (bodies) per second of the whole job; "
                           "achieved_GBs: compulsory HBM bytes per iteration in the streamed "
                           "formats (all ranks) x iterations/s",
            "achieved_GBs": round(value, 2),
            "bytes_per_iteration": iter_global,
            "iteration_frac": round(value / (HBM_PEAK_GBS * world), 4),
            "csr_equivalent_GBs": round(csr_eq, 2),
            "csr_equivalent_bytes_per_iteration": b_alg(n_global, nnz_global),
            "config": {"workload": workload + ", CSR fp64/int32 input, SpMV in the "
                                              "per-matrix best format",
                       "workload_id": args.workload,
                       "rows_global": n_global, "nnz_global": nnz_global,
                       "parallelism": f"rows{world}" if world > 1 else "single",
                       "transport": transport,
                       "peer_fallback_reason": peer_note,
                       "peer_form": peer_form,
                       "rccl_note": rccl_note,
                       "rccl_iteration": rccl_iteration,
                       "transport_validation": validation,
                       "iteration": {1: "3 kernels", 2: "fused (2 kernels)",
                                     3: "3 kernels, x update deferred over 4 bodies",
                                     4: ("3 launches (interior walk forming p_k with the halo "
                                         "push in front, boundary rows, update_r with both "
                                         "all-reduces), x update deferred over 4 bodies"
                                         if dist_on and world > 1 else
                                         "2 kernels (p update in the SpMV), x update deferred "
                                         "over 4 bodies"),
                                     5: "persistent body (one launch per chunk of bodies, two "
                                        "grid-wide exchanges per body)",
                                     6: "3 kernels, Ap recomputed (the walk's p.Ap; the walk "
                                        "again with r -= alpha A p; the p update), x update "
                                        "deferred over 4 bodies",
                                     7: "2 kernels, p update in the first walk and Ap "
                                        "recomputed (the tile walk forming p_k with p.Ap; the "
                                        "walk again with r -= alpha A p_k and the stop rule), "
                                        "x update deferred over 4 bodies (+ a flush launch in "
                                        "slot 3)"}[mode_eff] +
                                    (" (auto)" if args.mode == 0 else ""),
                       "setup": setup,
                       "spmv_variant": int(variant.value),
                       "spmv_autotune": autotune,
                       "value_code_templates": (
                           {"templates": ntpl.value, "slices": tpl_slices.value,
                            "slices_total": (n_local + 127) // 128,
                            "in_use": bool(variant.value & 8388608)}
                           if ntpl.value else None),
                       "lean_walk": (
                           {"classes": lean[0].value, "slices": lean[1].value,
                            "slices_total": (n_local + 127) // 128, "grid": lean[2].value,
                            "D": lean[3].value, "a": lean[4].value,
                            "chunked_walk": bool(lean[5].value), "in_use": lean_on,
                            "team_form": bool(team.value)}
                           if lean[0].value else None)},
            "roofline": roof,
            "csr_general": general,
            "cpu_baseline": cpu,
        }
    check(L.cgx_cg_destroy(cg))
    check(L.cgx_csr_destroy(A))
    if line is not None:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def coop_roofline(L, cg, avg, calls, bodies: int, iter_bytes: int) -> dict:
    """Mode 5 runs the whole body in one persistent kernel (k_cg_coop_wt or
    _tg), so the kernel's line is the iteration's: compulsory bytes of a
    body (as mode 1 moves them) over the HIP-event time per body. The body
    is latency-bound (two grid-wide exchanges, one gather round trip); its
    vectors stay in the L2s and the Infinity Cache, so no HBM traffic is
    claimed (PMC FETCH_SIZE would count the exchanges' L2-bypassing loads)."""
    from conjugategradient_amd._native import check

    R, NT, G, T = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    check(L.cgx_cg_coop_shape(cg, C.byref(R), C.byref(NT), C.byref(G), C.byref(T)))
    t_launch = avg[1] * 1e-3
    t_body = t_launch * calls[1] / max(bodies, 1)
    ach = iter_bytes / t_body / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": f"k_cg_coop_{'st' if T.value == 2 else 'wt'}",
            "template": f"<{R.value}, {NT.value}>", "workgroups": G.value,
            "bytes_per_launch": int(iter_bytes * bodies / max(calls[1], 1)),
            "bytes_basis": "compulsory bytes of a body as the three-kernel body moves them "
                           "(matrix stream + 16 n SpMV + 64 n updates) x bodies per launch",
            "avg_us": round(avg[1] * 1e3, 2), "launches_timed": int(calls[1]),
            "us_per_body": round(t_body * 1e6, 3),
            "traffic_note": "latency-bound persistent body: vectors L2 / Infinity-Cache "
                            "resident, no HBM traffic claimed"}


def kernel_base_name(full: str) -> str:
    """'void cgx::(anonymous namespace)::k_x<double, 5>(args...)' -> 'k_x<double, 5>'."""
    name = full.replace("(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "").replace("cgx::", "").strip()


def pmc_accumulate(f, ctr: str, sums: dict) -> None:
    """Add one rocprofv3 counter_collection.csv (open file) to sums[kernel][ctr]
    = [total, dispatches]."""
    import csv

    for r in csv.DictReader(f):
        if r.get("Counter_Name") != ctr:
            continue
        acc = sums.setdefault(kernel_base_name(r["Kernel_Name"]), {}).setdefault(ctr, [0.0, 0])
        acc[0] += float(r["Counter_Value"])
        acc[1] += 1


def pmc_bytes(sums: dict) -> dict:
    """HBM bytes per dispatch per kernel: (2 FETCH_SIZE + WRITE_SIZE) KB x 1024."""
    out = {}
    for name, c in sums.items():
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            f = c["FETCH_SIZE"][0] / c["FETCH_SIZE"][1]
            w = c["WRITE_SIZE"][0] / c["WRITE_SIZE"][1]
            out[name] = int(round((2 * f + w) * 1024))
    return out


def pmc_traffic(args, variant: str, mode: int, team: int = 0, timeout_s: float = 180.0) -> dict:
    """HBM bytes per launch of every kernel of the iteration, from two
    rocprofv3 PMC passes (FETCH_SIZE, then WRITE_SIZE: one counter group per
    run, kernel dispatch counters only) of a short child run of this same
    workload with the same SpMV variant and iteration mode. FETCH_SIZE is
    doubled (gfx950 tallies 128-B requests at 64 B; MI355X_MICROARCH.md,
    HBM/rocprofv3 section); KB = 1024 B. The child starts as a new process
    (this one has initialised the GPU: no exec), in its own process group,
    killed whole on timeout."""
    import glob
    import shutil
    import signal
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return {"error": "rocprofv3 not found"}
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--workload", args.workload,
             "--steps", "10", "--warmup", "2", "--profile-steps", "0", "--no-cpu",
             "--no-general", "--no-traffic", "--mode", str(mode), "--poll", str(args.poll),
             "--lean-team", str(int(team))]
    if args.grid:
        child += ["--grid", str(args.grid)]
    env = dict(os.environ, CGX_SPMV_VARIANT=variant)
    env.pop("WORLD_SIZE", None)
    sums: dict = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="cgx_pmc_")
        try:
            p = subprocess.Popen([prof, "--pmc", ctr, "-d", d, "-o", "run", "--output-format", "csv",
                                  "--"] + child, env=env, stdout=subprocess.DEVNULL,
                                 stderr=subprocess.PIPE, text=True, start_new_session=True)
            try:
                _, err = p.communicate(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.communicate()
                return {"error": f"rocprofv3 --pmc {ctr} timed out after {timeout_s:.0f} s"}
            if p.returncode != 0:
                return {"error": f"rocprofv3 --pmc {ctr} exited {p.returncode}: {err[-400:]}"}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                pmc_accumulate(open(f), ctr, sums)
        finally:
            shutil.rmtree(d, ignore_errors=True)
    return {"by_kernel": pmc_bytes(sums),
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate child runs of "
                      "this workload, 2 + 10 bodies, same variant and mode), mean per dispatch; "
                      "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 FETCH_SIZE "
                      "correction, MI355X_MICROARCH.md)"}


def validate_peer(L, q, world, rank, dist, nxy=48, planes=8, tol=1e-8, mode=0):
    """Solve a small slab problem (nxy x nxy x planes*world, `planes` z-planes
    per rank, b_i = i + 1, x0 = 0) twice on this node: over the device peer
    transport and over the context's setup transport (RCCL; the host
    transport in the one-GPU rehearsal). The peer transport passes when both solves
    converge (accuracy() < 1e-20), their body counts agree within 2, and
    their x agree to 1e-10 relative (SURVEY §8(c) tolerances). Collective;
    every rank returns the same verdict. mode 4: the peer solve runs the
    partitioned mode 4 (its kernels, with the lean interior walk forced)."""
    import numpy as np
    import torch

    import conjugategradient_amd as cga
    from conjugategradient_amd._native import F64, check

    nz = planes * world
    n_local = nxy * nxy * planes
    begin = rank * n_local
    nnz = L.cgx_poisson_nnz(3, nxy, nxy, nz, begin, begin + n_local)
    rows = cga.DeviceArray(q, n_local + 1, np.int32)
    cols = cga.DeviceArray(q, nnz, np.int32)
    vals = cga.DeviceArray(q, nnz, np.float64)
    b = cga.DeviceArray(q, n_local, np.float64)
    check(L.cgx_iota(q.handle, F64, b.ptr, n_local, float(begin)))
    out, xs = {}, {}
    why = None
    for name in ("peer", "setup"):
        # cgx_csr_create_dist remaps the columns in place (global -> local +
        # ghost numbering): every matrix gets freshly generated arrays
        check(L.cgx_poisson_fill(q.handle, F64, 3, nxy, nxy, nz, begin, begin + n_local,
                                 rows.ptr, cols.ptr, vals.ptr))
        A = C.c_void_p()
        check(L.cgx_csr_create_dist(q.handle, n_local * world, begin, n_local, nnz, rows.ptr,
                                    cols.ptr, vals.ptr, F64, C.byref(A)))
        try:
            if name == "peer":
                ok = C.c_int(0)
                check(L.cgx_dist_peer_enable(A, C.byref(ok)))
                if not ok.value:
                    why = "peer self-test: " + L.cgx_last_error().decode()
                    out[name] = {"enabled": False}
                    continue
            x = cga.DeviceArray(q, n_local, np.float64)
            x.fill(0.0)
            cg = C.c_void_p()
            rc = 0
            if name == "peer" and mode == 4:
                rc = L.cgx_csr_set_variant(A, KVL)
            check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
            if rc == 0 and name == "peer" and mode == 4:
                rc = L.cgx_cg_set_mode(cg, 4)
            bodies, rxr, acc = C.c_int64(), C.c_double(), C.c_double()
            if rc == 0:
                rc = L.cgx_cg_solve(cg, b.ptr, x.ptr, tol, -1, C.byref(bodies), C.byref(rxr))
            if rc == 0:
                check(L.cgx_accuracy(q.handle, A, b.ptr, x.ptr, C.byref(acc)))
                xs[name] = x.download()
                out[name] = {"bodies": int(bodies.value), "accuracy": float(acc.value)}
            else:
                why = f"{name} solve failed: " + L.cgx_last_error().decode()
                out[name] = {"error": why}
            L.cgx_cg_destroy(cg)
        finally:
            L.cgx_csr_destroy(A)
    ok_local = "peer" in xs and "setup" in xs
    d2 = r2 = 0.0
    if ok_local:
        d2 = float(np.sum((xs["peer"] - xs["setup"]) ** 2))
        r2 = float(np.sum(xs["setup"] ** 2))
    t = torch.tensor([d2, r2, 0.0 if ok_local else 1.0], dtype=torch.float64)
    dist.all_reduce(t)
    rel = math.sqrt(t[0].item() / t[1].item()) if t[1].item() > 0 else float("inf")
    ok = t[2].item() == 0.0
    if ok:
        p, r = out["peer"], out["setup"]
        ok = (abs(p["bodies"] - r["bodies"]) <= 2 and p["accuracy"] < 1e-20
              and r["accuracy"] < 1e-20 and rel <= 1e-10)
        if not ok:
            why = f"peer and setup-transport solves disagree: {out}, rel {rel:.3e}"
    # every rank's verdict (accuracy and bodies are global: the same on all)
    v = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64)
    dist.all_reduce(v)
    ok = v.item() == 0.0
    if not ok and why is None:
        why = "another rank's validation failed"
    return {"ok": bool(ok), "grid": [nxy, nxy, nz], "tol": tol, "solves": out,
            "x_rel_peer_vs_setup": rel, "why": why, "peer_mode": mode or "auto"}


def general_formats(L, q, A, b, x, n, nnz, mode_eff, args, steps=100, prof=50):
    """The same matrix with value codes off: plain SELL-P (8 B of value per
    slot, the format of a banded matrix with many distinct values) and
    CSR-stream (the general CSR kernel: any sparsity, e.g. G3_circuit).
    Per format: iterations/s over `steps` graph-replayed bodies, and the
    SpMV's HIP-event time priced at its own format's compulsory bytes."""
    from conjugategradient_amd._native import check

    out = {}
    orig = C.c_int(0)
    check(L.cgx_csr_variant(A, C.byref(orig)))
    # (mode 6 recomputes Ap with the lean walk; the general formats run its
    # stored-Ap body, mode 3)
    mode_eff = 3 if mode_eff in (6, 7) else mode_eff
    for name, req in (("sellp_plain", 8194), ("csr_stream", 15)):
        try:
            check(L.cgx_csr_set_variant(A, req))
        except Exception as e:  # the matrix lacks the layout
            out[name] = {"error": str(e)}
            continue
        v = C.c_int(0)
        check(L.cgx_csr_variant(A, C.byref(v)))
        sb = C.c_int64(0)
        check(L.cgx_csr_stream_bytes(A, C.byref(sb)))
        cg = C.c_void_p()
        check(L.cgx_cg_create(q.handle, A, C.byref(cg)))
        check(L.cgx_cg_config(cg, args.poll, 1))
        check(L.cgx_cg_set_mode(cg, mode_eff))
        check(L.cgx_cg_begin(cg, b.ptr, x.ptr, 0.0, 10 + steps + prof))
        bodies, stopped = C.c_int64(0), C.c_int(0)
        check(L.cgx_cg_run(cg, 10, C.byref(bodies), C.byref(stopped)))
        q.wait()
        t0 = time.perf_counter()
        check(L.cgx_cg_run(cg, steps, C.byref(bodies), C.byref(stopped)))
        q.wait()
        t1 = time.perf_counter()
        avg = (C.c_double * 4)()
        calls = (C.c_int64 * 4)()
        check(L.cgx_cg_set_kernel_timing(cg, 1))
        check(L.cgx_cg_run(cg, prof, C.byref(bodies), C.byref(stopped)))
        if hasattr(L, "cgx_cg_kernel_exec_times"):
            check(L.cgx_cg_kernel_exec_times(cg, avg, calls))
        if calls[1] == 0:
            check(L.cgx_cg_kernel_times(cg, avg, calls))
        check(L.cgx_cg_destroy(cg))
        its = steps / (t1 - t0)
        kb = spmv_bytes_per_iter(sb.value, n, mode_eff)
        it_b = kb + update_bytes_per_iter(n, mode_eff)
        out[name] = {"spmv_variant": int(v.value), "iterations_per_s": round(its, 2),
                     "GBs": round(it_b * its / 1e9, 1),
                     "iteration_frac": round(it_b * its / 1e9 / HBM_PEAK_GBS, 4),
                     "spmv_avg_us": round(avg[1] * 1e3, 2), "spmv_bytes_per_launch": kb,
                     "spmv_frac": round(kb / (avg[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "csr_equivalent_spmv_frac": round(
                         csr_spmv_bytes(n, nnz) / (avg[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    check(L.cgx_csr_set_variant(A, orig.value))
    return out


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rc = maybe_launch(args, argv)
    if rc is not None:
        return rc
    run(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
