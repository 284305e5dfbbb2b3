"""Every VectorOperations method of the C++ drop-in header
(include/VectorOperations.hpp), called from C++ with device Scalars the way
the reference's callers do (src/VectorOperations.hpp:110-466,
src/CG.hpp:364-418), checked against the oracle.

examples/vecops_check.cpp reads the inputs the test writes and writes every
result back:
  * dot_product_optimised (:110-208), dot_product (:212-285),
    dot_product_trivial (:287-309) and norm (:311-331) ACCUMULATE onto a
    non-zero initial scalar (Q4); reductions run in another order than the
    oracle's index order, so they are held to 1e-13 relative;
  * saxpby (:349-367), sambx (:380-397), sapbx (:410-428, also in place),
    spmv (:438-466, with `count`) are bit-exact (products rounded before the
    add in both, -ffp-contract=off).
"""
import os
import subprocess

import numpy as np
import pytest

from tests.util import irregular_spd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "examples", "vecops_check")


def test_vecops_check_compiles(tmp_path):
    out = str(tmp_path / "vecops_check")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "examples", "vecops_check.cpp"), "-o", out,
                        "-L" + os.path.join(ROOT, "conjugategradient_amd"), "-lcgx",
                        "-Wl,-rpath," + os.path.join(ROOT, "conjugategradient_amd")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1000, 300_001])
def test_vector_operations_header_against_oracle(oracle, tmp_path, n):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], check=True)
    rp, cl, vl = irregular_spd(n, seed=7)
    rng = np.random.default_rng(n)
    x, y = rng.standard_normal(n), rng.standard_normal(n)
    a, b, r0 = 0.75, -1.25, 1.5
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(inp, "wb") as f:
        np.array([n, len(vl)], np.int64).tofile(f)
        rp.astype(np.int32).tofile(f)
        cl.astype(np.int32).tofile(f)
        vl.astype(np.float64).tofile(f)
        x.tofile(f)
        y.tofile(f)
        np.array([a, b, r0], np.float64).tofile(f)
    p = subprocess.run([EXE, str(inp), str(out)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    res = np.fromfile(out, np.float64)
    assert res.size == 4 + 5 * n
    dots = res[:4]
    want_dot = oracle.dot_acc(x, y, r0)
    for got in dots[:3]:
        assert got == pytest.approx(want_dot, rel=1e-13, abs=1e-13 * np.abs(x * y).sum())
    assert dots[3] == pytest.approx(oracle.norm_acc(x, r0), rel=1e-13)
    v = res[4:].reshape(5, n)
    np.testing.assert_array_equal(v[0], oracle.saxpby(x, y, a, b))
    np.testing.assert_array_equal(v[1], oracle.sambx(x, y, b))
    np.testing.assert_array_equal(v[2], oracle.sapbx(x, y, b))
    np.testing.assert_array_equal(v[3], oracle.spmv(rp, cl, vl, x))
    np.testing.assert_array_equal(v[4], oracle.sapbx(x, y, b))
