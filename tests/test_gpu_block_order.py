"""CSR-stream's row-block visit order (cgx_csr_set_block_order):
the blocks of each XCD eighth walked in chunks of a plane through the planes.
Every row's sum is unchanged (a block sums its rows exactly as in the
natural order), so Ap must equal the oracle's per-row loop (CG.hpp's
VectorOperations::spmv, VectorOperations.hpp:438-466) bit for bit in every
CSR-stream form, and CG over it must match the oracle's iterates.
"""
import ctypes as C

import numpy as np
import pytest

from conjugategradient_amd import CG, Matrix, Vector, VectorOperations
from conjugategradient_amd._native import CgxError, check, lib
from tests.util import irregular_spd, rel

pytestmark = pytest.mark.gpu


def order_info(m):
    d, w = C.c_int(), C.c_int()
    check(lib().cgx_csr_block_order_info(m.schedule(), C.byref(d), C.byref(w)))
    return d.value, w.value


def spmv(queue, m, x):
    n = m.N()
    ops = VectorOperations(queue, np.float64)
    ops.setVectorSize(n)
    y = Vector(queue, n)
    ops.spmv(m, Vector(queue, x), y, m.NNZ(), count=n)
    return y.to_numpy()


@pytest.mark.parametrize("variant", [15, 13, 5, 265])
@pytest.mark.parametrize("chunk", [256, 1024, -1])
def test_block_order_spmv_bitexact(queue, oracle, variant, chunk):
    rp, cl, vl = oracle.poisson(3, 64, 64, 64)
    n = len(rp) - 1
    rng = np.random.default_rng(5)
    vl = vl * rng.uniform(0.5, 1.5, len(vl))  # many distinct values: CSR's domain
    m = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_variant(m.schedule(), variant))
    check(lib().cgx_csr_set_block_order(m.schedule(), chunk))
    d, w = order_info(m)
    if chunk > 0:
        assert (d, w) == (4096, chunk)
    else:  # 64^3: two planes of stream fit half an L2, no order
        assert (d, w) == (0, 0)
    x = rng.standard_normal(n)
    x[[0, 4095, 4096, n // 2, n - 1]] = [np.inf, -0.0, np.nan, 0.0, -0.0]
    np.testing.assert_array_equal(spmv(queue, m, x), oracle.spmv(rp, cl, vl, x))


def test_block_order_auto_at_128cubed(queue, oracle):
    rp, cl, vl = oracle.poisson(3, 128, 128, 128)
    n = len(rp) - 1
    m = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_variant(m.schedule(), 15))
    check(lib().cgx_csr_set_block_order(m.schedule(), -1))
    d, w = order_info(m)
    assert d == 16384 and w > 0 and w % 256 == 0
    x = np.random.default_rng(2).standard_normal(n)
    np.testing.assert_array_equal(spmv(queue, m, x), oracle.spmv(rp, cl, vl, x))
    b = np.arange(1, n + 1, dtype=np.float64)  # Tester.cpp:27-30
    cg = CG(queue)
    cg.mode = 3
    cg.setMatrix(m)
    cg.setTarget(b)
    cg.solve(0.0, max_iter=20)
    _, xr = oracle.cg_fixed_iters_omp(rp, cl, vl, b, 20, 8)
    assert rel(cg.extract(), xr) <= 1e-10


def test_block_order_refused_without_a_plane_offset(queue):
    rp, cl, vl = irregular_spd(20000, mean_deg=4.0, seed=3)
    m = Matrix(queue, vl, cl, rp)
    with pytest.raises(CgxError, match="dominant plane offset"):
        check(lib().cgx_csr_set_block_order(m.schedule(), 1024))
    check(lib().cgx_csr_set_block_order(m.schedule(), -1))  # automatic: natural order
    assert order_info(m) == (0, 0)
