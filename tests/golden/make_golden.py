#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ (run in the build
container, where /root/reference exists).

* poisson*.mtx — lower-triangle `symmetric` Matrix-Market files with one
  comment line, written by the oracle's emitter.
* quirks_*.mtx — inputs that exercise the reference loader's quirks: no
  comment line (Q1: line 2 is dropped), a `general` banner (Q2: mirrored
  anyway), an empty row (Q3: dropped from rowptr), unsorted entries.
* loader_<name>.npz — rowptr/col/val as returned by the REFERENCE's own
  read_file (test/mm_reader.cpp compiled unmodified into
  oracle/_ref/libmmref.so): the loader golden vectors.
* cg_<name>.npz — the oracle's CG::solve restatement on b_i = i + 1:
  x and the loop-body counts at tol 1e-8 and 1e-24, accuracy(). The counts
  are the reference-probe values recorded in SURVEY §6/§8(c) (103, 972, 479,
  152, 76); the oracle reproduces them exactly, which is what pins it.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

POISSON = {"poisson2d_16": (2, 16, 16, 1), "poisson2d_128": (2, 128, 128, 1),
           "poisson3d_16": (3, 16, 16, 16)}

QUIRKS = {
    # Q1: no comment line -> the size line is dropped, the first entry line is
    # taken as the size line and its entry is lost
    "quirks_nocomment": "%%MatrixMarket matrix coordinate real symmetric\n"
                        "4 4 6\n1 1 4.0\n2 1 -1.0\n2 2 4.0\n3 3 4.0\n4 3 -1.0\n4 4 4.0\n",
    # Q2: `general` banner, off-diagonals are mirrored anyway; unsorted input
    "quirks_general": "%%MatrixMarket matrix coordinate real general\n% c\n"
                      "3 3 4\n3 3 2.5\n1 1 2.0\n2 1 -0.5\n2 2 3.0\n",
    # Q3: row 2 (1-based) has no entry -> it vanishes from rowptr
    "quirks_emptyrow": "%%MatrixMarket matrix coordinate real symmetric\n% c\n% c2\n"
                       "4 4 3\n1 1 1.0\n3 3 2.0\n4 4 3.0\n",
}


def main() -> None:
    if not O.ref_available():
        O.build(ref=True)
    for name, (dim, nx, ny, nz) in POISSON.items():
        rp, cl, vl = O.poisson(dim, nx, ny, nz)
        path = os.path.join(HERE, name + ".mtx")
        O.write_mtx_lower(path, rp, cl, vl)
        ref = O.ref_read_mtx(path)
        np.savez_compressed(os.path.join(HERE, f"loader_{name}.npz"), rowptr=ref[0],
                            col=ref[1], val=ref[2])
        b = np.arange(1, len(rp), dtype=np.float64)
        out = {}
        for tag, tol in (("1e-8", 1e-8), ("1e-24", 1e-24)):
            x, res = O.cg_solve(rp, cl, vl, b, tol)
            out[f"x_{tag}"] = x
            out[f"iters_{tag}"] = np.int64(res.iterations)
            out[f"accuracy_{tag}"] = np.float64(O.accuracy(rp, cl, vl, b, x))
        np.savez_compressed(os.path.join(HERE, f"cg_{name}.npz"), **out)
        print(name, {k: v for k, v in out.items() if not k.startswith("x_")})
    for name, text in QUIRKS.items():
        path = os.path.join(HERE, name + ".mtx")
        with open(path, "w") as f:
            f.write(text)
        ref = O.ref_read_mtx(path)
        np.savez_compressed(os.path.join(HERE, f"loader_{name}.npz"), rowptr=ref[0],
                            col=ref[1], val=ref[2])
        print(name, ref)


if __name__ == "__main__":
    main()
