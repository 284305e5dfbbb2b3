"""CPU emulation of libcgx's multi-GPU CG (cgx_dist.cpp) over torch.distributed
gloo: the same contiguous row partition, the same halo plan (built by
libcgx's own host helpers cgx_plan_ghosts / cgx_plan_remap), the same
per-iteration exchange points (halo of p before the SpMV, all-reduce of p.Ap
and of r.r) and the same stop rule. Used by tests/test_dist_cpu.py.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from conjugategradient_amd._native import lib


def partition(n: int, world: int):
    base, extra = divmod(n, world)
    counts = np.array([base + (r < extra) for r in range(world)], np.int64)
    begins = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    return begins, counts


def build_plan(rank, world, rp, cl):
    """Local CSR with local/ghost column numbering + halo plan."""
    L = lib()
    n = len(rp) - 1
    begins, counts = partition(n, world)
    a, b = int(begins[rank]), int(begins[rank] + counts[rank])
    lrp = (rp[a:b + 1] - rp[a]).astype(np.int32)
    lcol = cl[rp[a]:rp[b]].astype(np.int32).copy()
    ng = C.c_int64()
    gp = C.POINTER(C.c_int64)()
    recv = np.zeros(world, np.int64)
    rc = L.cgx_plan_ghosts(counts[rank], a, len(lcol), lcol.ctypes.data, world,
                           begins.ctypes.data, counts.ctypes.data, C.byref(ng), C.byref(gp),
                           recv.ctypes.data)
    assert rc == 0
    ghosts = np.ctypeslib.as_array(gp, shape=(max(ng.value, 1),))[:ng.value].copy()
    rc = L.cgx_plan_remap(counts[rank], a, len(lcol), lcol.ctypes.data, ng.value, gp)
    assert rc == 0
    L.cgx_free_host(C.cast(gp, C.c_void_p))
    # requests: ghosts grouped by owner (sorted ids => owner order)
    req = {}
    off = 0
    for r in range(world):
        if recv[r]:
            req[r] = ghosts[off:off + recv[r]]
            off += recv[r]
    everyone = [None] * world
    dist.all_gather_object(everyone, {r: v.tolist() for r, v in req.items()})
    send = {}
    for r in range(world):
        if r != rank and rank in everyone[r]:
            ids = np.array(everyone[r][rank], np.int64)
            assert np.all((ids >= a) & (ids < b))
            send[r] = (ids - a).astype(np.int64)
    recv_off = {}
    off = 0
    for r in range(world):
        if r in req:
            recv_off[r] = (off, len(req[r]))
            off += len(req[r])
    return dict(a=a, b=b, n_local=b - a, rowptr=lrp, col=lcol, ghosts=ghosts, send=send,
                recv=recv_off)


def halo(plan, v_ext):
    """Fill v_ext's ghost area (the ncclSend/ncclRecv group of
    dist_halo_exchange)."""
    nl = plan["n_local"]
    reqs = []
    bufs = {}
    for r, idx in plan["send"].items():
        reqs.append(dist.isend(torch.from_numpy(v_ext[idx].copy()), r))
    for r, (off, cnt) in plan["recv"].items():
        bufs[r] = torch.empty(cnt, dtype=torch.float64)
        reqs.append(dist.irecv(bufs[r], r))
    for q in reqs:
        q.wait()
    for r, (off, cnt) in plan["recv"].items():
        v_ext[nl + off: nl + off + cnt] = bufs[r].numpy()


def allreduce(v: float) -> float:
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t)
    return float(t.item())


def _two_sum_into(s, x):
    """s = [hi, lo] += x (TwoSum, cgx_dd.h Dd::operator+=)."""
    hi = s[0]
    t = hi + x
    z = t - hi
    s[1] += (hi - (t - z)) + (x - z)
    s[0] = t


def dd_dot(a, b):
    """This rank's double-length sum of the rounded products a_i b_i."""
    s = [0.0, 0.0]
    for x in (np.asarray(a) * np.asarray(b)).tolist():
        _two_sum_into(s, x)
    return s


def dd_allreduce(pair) -> float:
    """The peer transport's world sum (cgx_peer_dev.h world_sum): every
    rank's pair, combined in rank order as pairs, rounded once."""
    pairs = [None] * dist.get_world_size()
    dist.all_gather_object(pairs, (float(pair[0]), float(pair[1])))
    s = [pairs[0][0], pairs[0][1]]
    for hi, lo in pairs[1:]:
        _two_sum_into(s, hi)
        s[1] += lo
    return s[0] + s[1]


def solve(plan, val_local, b_local, tol, oracle, n_global, dots="plain"):
    """libcgx's iteration (k_spmv_dot / k_update_r / k_update_xp) with the
    reference's stop rule; returns (x_local, bodies). dots="dd": every dot a
    double-length sum per rank and a pair world sum (round 6's engine)."""
    if dots == "dd":
        def gdot(u, v):
            return dd_allreduce(dd_dot(u, v))
    else:
        def gdot(u, v):
            return allreduce(oracle.dot_acc(u, v, 0.0))
    nl = plan["n_local"]
    ng = len(plan["ghosts"])
    rp, cl = plan["rowptr"], plan["col"]
    x = np.zeros(nl)
    xe = np.zeros(nl + ng)
    halo(plan, xe)
    r = b_local - oracle.spmv(rp, cl, val_local, xe)
    p = np.zeros(nl + ng)
    p[:nl] = r
    rxr = gdot(r, r)
    bodies = 0
    cap = n_global + 1
    while True:
        halo(plan, p)
        Ap = oracle.spmv(rp, cl, val_local, p)
        pAp = gdot(Ap, p[:nl])
        alpha = rxr / pAp
        r = oracle.sambx(r, Ap, alpha)
        rr = gdot(r, r)
        beta = rr / rxr
        x = oracle.sapbx(x, p[:nl], alpha)
        p[:nl] = oracle.sapbx(r, p[:nl], beta)
        bodies += 1
        stop = np.isnan(rxr) or np.sqrt(rxr) <= tol
        rxr = rr
        if stop or bodies >= cap:
            return x, bodies
