"""World-size-2 (and 3) gloo run of the row-partitioned CG on CPU: the halo
plan from libcgx's host helpers + the distributed iteration reproduce the
single-process oracle solve (x within 1e-10, bodies within 2)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, out):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from tests import dist_emul as D
        from tests.util import irregular_spd

        if case == "poisson3d":
            rp, cl, vl = O.poisson(3, 10, 9, 14)
            tol = 1e-8
        elif case == "slabs":  # 2 planes per rank at world 8
            rp, cl, vl = O.poisson(3, 8, 8, 16)
            tol = 1e-8
        else:
            rp, cl, vl = irregular_spd(4000, seed=21, shift=1.0)
            tol = 1e-8
        n = len(rp) - 1
        plan = D.build_plan(rank, world, rp, cl)
        b = np.arange(1, n + 1, dtype=np.float64)
        a, e = plan["a"], plan["b"]
        x, bodies = D.solve(plan, vl[rp[a]:rp[e]], b[a:e], tol, O, n)
        parts = [None] * world
        dist.all_gather_object(parts, x.tolist())
        nb = [None] * world
        dist.all_gather_object(nb, (len(plan["ghosts"]), bodies))
        if rank == 0:
            out.put((np.concatenate([np.array(p) for p in parts]), bodies,
                     len(plan["ghosts"]), nb))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [(2, "poisson3d"), (3, "poisson3d"), (2, "irregular"),
                                        (8, "slabs")])
def test_distributed_cg_matches_single_process(oracle, world, case):
    """World 8 is config 4's split (BASELINE.json configs[3]): a 8 x 8 x 16 grid
    in 2-plane slabs, 6 inner ranks with two neighbours and 2 end ranks."""
    from tests.util import irregular_spd, rel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(world, _free_port(), case, q), nprocs=world,
                       start_method="spawn", join=True)
    x, bodies, ghosts, per_rank = q.get(timeout=120)
    # the ranks agree on the stop (every rank derives the same scalars)
    assert len({b for _, b in per_rank}) == 1, per_rank
    if case == "poisson3d":
        rp, cl, vl = oracle.poisson(3, 10, 9, 14)
    elif case == "slabs":
        rp, cl, vl = oracle.poisson(3, 8, 8, 16)
        assert [g for g, _ in per_rank] == [64] + [128] * 6 + [64], per_rank
    else:
        rp, cl, vl = irregular_spd(4000, seed=21, shift=1.0)
    b = np.arange(1, len(rp), dtype=np.float64)
    xr, res = oracle.cg_solve(rp, cl, vl, b, 1e-8)
    assert ghosts > 0
    assert abs(bodies - res.iterations) <= 2
    assert rel(x, xr) <= 1e-10


def _dd_worker(rank, world, port, out):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from tests import dist_emul as D

        rp, cl, vl = O.poisson(3, 8, 8, 16)
        n = len(rp) - 1
        plan = D.build_plan(rank, world, rp, cl)
        b = np.arange(1, n + 1, dtype=np.float64)
        a, e = plan["a"], plan["b"]
        x, bodies = D.solve(plan, vl[rp[a]:rp[e]], b[a:e], 1e-8, O, n, dots="dd")
        parts = [None] * world
        dist.all_gather_object(parts, x.tolist())
        if rank == 0:
            out.put((np.concatenate([np.array(p) for p in parts]), bodies))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_distributed_dd_dots_bit_identical_to_dd_oracle(oracle, world):
    """Round 6's dots (double-length sums per rank, the ranks' pairs summed in
    rank order and rounded once, as cgx_peer_dev.h world_sum) make the
    partitioned solve independent of the world size: at 1, 2, 3 and 8 ranks
    the bodies and x equal oracle.cg_solve_dd's bit for bit (the GPU's x is
    held to the same oracle in tests/test_gpu_determinism.py and
    test_gpu_dist.py::test_partitioned_x_independent_of_world_size)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_dd_worker, args=(world, _free_port(), q), nprocs=world,
                       start_method="spawn", join=True)
    x, bodies = q.get(timeout=120)
    rp, cl, vl = oracle.poisson(3, 8, 8, 16)
    b = np.arange(1, len(rp), dtype=np.float64)
    xr, res = oracle.cg_solve_dd(rp, cl, vl, b, 1e-8, threads=4)
    assert bodies == res.iterations
    assert np.array_equal(x, xr)
