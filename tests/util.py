"""Deterministic test inputs (numpy only; no reference code)."""
from __future__ import annotations

import numpy as np


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


def rel(a, b) -> float:
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(b))
