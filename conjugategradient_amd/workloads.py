"""The BASELINE.json configurations as matrices in HBM.

  p3d_256     3-D 7-point Dirichlet Poisson 256^3 (the headline config)
  p3d_512     3-D 7-point Poisson 512^3 (config 4; z-slabs over the ranks)
  p2d_4096    2-D 5-point Poisson 4096^2
  p2d_128     2-D 5-point Poisson 128^2, read from tests/golden/poisson2d_128.mtx
              through the Matrix-Market loader (config 1's input path)
  g3_standin  the G3_circuit stand-in: a seeded irregular SPD random-graph
              Laplacian with N = 1,585,478 rows (G3_circuit is not available
              offline)

The Poisson matrices are generated on the device (cgx_poisson_fill), rows
in natural order, columns ascending (what mm_reader.cpp:76-86 produces for
the same .mtx). b_i = i + 1 (Tester.cpp:27-30), x0 = 0.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

G3_ROWS = 1_585_478  # G3_circuit's row count (SuiteSparse metadata)
G3_MEAN_DEG = 3.83   # couplings per row: ~4.8 entries per row with the diagonal

# name: (dim, nx, ny, nz) for the device generator; None for host-built inputs
POISSON = {"p3d_256": (3, 256, 256, 256), "p3d_512": (3, 512, 512, 512),
           "p2d_4096": (2, 4096, 4096, 1)}
WORKLOADS = ("p3d_256", "p3d_512", "p2d_4096", "p2d_128", "g3_standin")


def coo_to_csr(n, rows, cols, vals):
    """Sum duplicates, sort by (row, col) -> (rowptr, col, val) int32/f64."""
    key = rows.astype(np.int64) * n + cols.astype(np.int64)
    order = np.argsort(key, kind="stable")
    key, vals = key[order], vals[order]
    uniq, start = np.unique(key, return_index=True)
    v = np.add.reduceat(vals, start)
    r = (uniq // n).astype(np.int64)
    c = (uniq % n).astype(np.int32)
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, r + 1, 1)
    rowptr = np.cumsum(rowptr).astype(np.int32)
    return rowptr, c, v.astype(np.float64)


def irregular_spd(n: int, mean_deg: float = 3.8, seed: int = 12345, hub: int = 0,
                  shift: float = 1e-2):
    """Random-graph Laplacian + diagonal shift: SPD with varied row lengths
    (the G3_circuit stand-in of SURVEY §8(d)). `hub` > 0 adds one vertex
    coupled to `hub` others (a row longer than one SpMV tile)."""
    rng = np.random.default_rng(seed)
    m = int(n * mean_deg / 2)
    a = rng.integers(0, n, m)
    # mostly-local couplings, like a circuit netlist in natural order
    off = rng.geometric(0.02, m) * rng.choice([-1, 1], m)
    b = np.clip(a + off, 0, n - 1)
    keep = a != b
    a, b = a[keep], b[keep]
    if hub:
        h = n // 2
        others = rng.choice(np.setdiff1d(np.arange(n), [h]), size=min(hub, n - 1), replace=False)
        a = np.concatenate([a, np.full(len(others), h)])
        b = np.concatenate([b, others])
    w = rng.uniform(0.5, 2.0, len(a))
    rows = np.concatenate([a, b])
    cols = np.concatenate([b, a])
    vals = np.concatenate([-w, -w])
    deg = np.zeros(n)
    np.add.at(deg, a, w)
    np.add.at(deg, b, w)
    rows = np.concatenate([rows, np.arange(n)])
    cols = np.concatenate([cols, np.arange(n)])
    vals = np.concatenate([vals, deg + shift])
    return coo_to_csr(n, rows, cols, vals)


@dataclass
class Slab:
    """One rank's rows of a workload, in HBM (int32 rowptr/col, f64 val)."""
    name: str
    description: str
    n_global: int
    nnz_global: int
    row_begin: int
    n_local: int
    nnz_local: int
    rows: object  # DeviceArray
    cols: object
    vals: object


def host_csr(name: str):
    """(rowptr, col, val) of a host-built workload (p2d_128, g3_standin)."""
    if name == "p2d_128":
        from .mtx import read_file
        data, cols, rows = read_file(os.path.join(ROOT, "tests", "golden", "poisson2d_128.mtx"))
        return (np.asarray(rows, np.int32), np.asarray(cols, np.int32),
                np.asarray(data, np.float64))
    if name == "g3_standin":
        return irregular_spd(G3_ROWS, mean_deg=G3_MEAN_DEG, seed=12345)
    raise ValueError(f"{name} is generated on the device")


def build(L, q, name: str, world: int = 1, rank: int = 0, grid: int | None = None,
          weak: bool = False) -> Slab:
    """Rank `rank`'s rows of workload `name` in HBM. Poisson workloads split
    into contiguous z-slabs (strong scaling: the global grid divided; weak:
    every rank an n^3 slab); the host-built ones run on one GPU only.
    `grid` overrides n of the 3-D workloads (bench.py --grid)."""
    from . import DeviceArray
    from ._native import F64, check

    if name in POISSON:
        dim, nx, ny, nz = POISSON[name]
        if grid and dim == 3:
            nx = ny = nz = grid
        if world > 1 and dim != 3:
            raise SystemExit(f"{name}: the multi-GPU split is for the 3-D workloads")
        if weak:
            nz_global = nz * world
            n_local = nx * ny * nz
        else:
            if nz % world:
                raise SystemExit(f"strong scaling needs the grid's z extent ({nz}) divisible by "
                                 f"the GPU count ({world})")
            nz_global = nz
            n_local = nx * ny * (nz // world)
        n_global = n_local * world
        row_begin = rank * n_local
        nnz_local = L.cgx_poisson_nnz(dim, nx, ny, nz_global, row_begin, row_begin + n_local)
        nnz_global = L.cgx_poisson_nnz(dim, nx, ny, nz_global, 0, n_global)
        rows = DeviceArray(q, n_local + 1, np.int32)
        cols = DeviceArray(q, nnz_local, np.int32)
        vals = DeviceArray(q, nnz_local, np.float64)
        check(L.cgx_poisson_fill(q.handle, F64, dim, nx, ny, nz_global, row_begin,
                                 row_begin + n_local, rows.ptr, cols.ptr, vals.ptr))
        if dim == 3:
            desc = (f"3D 7-pt Poisson {nx}^3 global, {nz_global // world} z-planes per GPU"
                    if not weak else
                    f"3D 7-pt Poisson {nx}^3 per GPU (global {nx}x{ny}x{nz_global})")
        else:
            desc = f"2D 5-pt Poisson {nx}^2"
        return Slab(name, desc, n_global, nnz_global, row_begin, n_local, nnz_local, rows, cols,
                    vals)
    if world > 1:
        raise SystemExit(f"{name}: a one-GPU workload")
    rp, cl, vl = host_csr(name)
    n, nnz = len(rp) - 1, len(vl)
    rows, cols, vals = DeviceArray(q, n + 1, np.int32), DeviceArray(q, nnz, np.int32), \
        DeviceArray(q, nnz, np.float64)
    rows.upload(rp)
    cols.upload(cl)
    vals.upload(vl)
    desc = {"p2d_128": "2D 5-pt Poisson 128^2 read from tests/golden/poisson2d_128.mtx "
                       "(cgx_mm_read, mm_reader.cpp semantics)",
            "g3_standin": f"G3_circuit stand-in: seeded irregular SPD, N = {n:,}, "
                          f"nnz = {nnz:,} (random-graph Laplacian + 1e-2 shift)"}[name]
    return Slab(name, desc, n, nnz, 0, n, nnz, rows, cols, vals)
