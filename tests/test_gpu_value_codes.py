"""SELL-P value codes (variant bit 32768) against the oracle.

A matrix with a SELL-P copy and at most 255 distinct values (bit patterns)
also gets one code byte per slot into a value dictionary; the kernel decodes
the stored value's exact bits, so the bar is bit-exactness with the oracle's
restatement of the reference SpMV (VectorOperations.hpp:438-466) and with the
plain SELL-P variant. Matrices with more distinct values keep plain values.
"""
import ctypes as C

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd import Matrix, Vector, VectorOperations
from conjugategradient_amd._native import CgxError, check, lib
from tests.test_gpu_sell import banded
from tests.util import rel

pytestmark = pytest.mark.gpu

# value codes: default / non-temporal loads; pipelined; pipelined with the
# +-1 neighbours from the adjacent lanes (bit 1048576)
VC = [34816, 34818, 559104, 559106, 1607680, 1607682]
VC4 = [296960, 296962, 821248, 821250, 1869824, 1869826]  # 4-bit codes (<= 15 values)
PLAIN = [8192, 8194, 13]     # SELL-P values, CSR-stream


def quantized_banded(n, levels, seed=5, rare=0):
    """banded() with values snapped to `levels` distinct numbers; `rare` > 0
    gives rows in the middle of the matrix values of their own (absent from
    the host's spread sample: the pack kernel's miss path adds them)."""
    rp, cl, vl = banded(n, half=4, seed=seed)
    grid = np.linspace(vl.min(), vl.max(), levels)
    vl = grid[np.clip(np.searchsorted(grid, vl), 0, levels - 1)]
    if rare:
        mid = n // 2 + 17
        for t in range(rare):
            vl[rp[mid + 3 * t]] = 1000.0 + t / 7.0
    return rp, cl, vl


def n_codes(m):
    nv = C.c_int()
    check(lib().cgx_csr_value_codes(m.schedule(), C.byref(nv)))
    return nv.value


def spmv_all(queue, A, x, variants, dtype=np.float64):
    n = A.N()
    ops = VectorOperations(queue, dtype)
    ops.setVectorSize(n)
    xv = Vector(queue, x, dtype=dtype)
    out = {}
    for v in variants:
        check(lib().cgx_csr_set_variant(A.schedule(), v))
        yv = Vector(queue, n, dtype=dtype)
        ops.spmv(A, xv, yv, A.NNZ(), count=n)
        out[v] = yv.to_numpy()
    return out


CASES = {
    "poisson2d": lambda O: O.poisson(2, 96, 80, 1),
    "poisson3d_ragged": lambda O: O.poisson(3, 23, 19, 17),
    "poisson3d_64": lambda O: O.poisson(3, 64, 64, 64),        # > sample size
    "quant200": lambda O: quantized_banded(60_001, 200),
    "quant_rare": lambda O: quantized_banded(60_001, 40, rare=20),
    "tiny": lambda O: (np.array([0, 1, 3, 4], np.int32), np.array([0, 0, 1, 2], np.int32),
                       np.array([2.0, -1.0, 3.0, 4.0])),
}
EXPECT_CODES = {"poisson2d": 2, "poisson3d_ragged": 2, "poisson3d_64": 2, "tiny": 4,
                "quant_rare": None, "quant200": None}


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_value_codes_bitexact(queue, oracle, case, dtype):
    rp, cl, vl = CASES[case](oracle)
    n = len(rp) - 1
    A = Matrix(queue, vl, cl, rp, dtype=dtype)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    nv = n_codes(A)
    distinct = len(np.unique(vl.astype(dtype).view(np.uint64 if dtype == np.float64
                                                   else np.uint32)))
    assert nv == distinct, (case, nv, distinct)
    if EXPECT_CODES[case] is not None:
        assert nv == EXPECT_CODES[case]
    x = np.random.default_rng(3).standard_normal(n)
    vc4 = VC4 if nv <= 15 else []
    if not vc4:
        with pytest.raises(CgxError, match="4-bit"):
            check(lib().cgx_csr_set_variant(A.schedule(), VC4[0]))
    out = spmv_all(queue, A, x, VC + vc4 + PLAIN, dtype)
    v = C.c_int()
    for set_v, want in ((34818, 40962), (296962, 303106)):
        if set_v in VC4 and not vc4:
            continue
        check(lib().cgx_csr_set_variant(A.schedule(), set_v))
        check(lib().cgx_csr_variant(A.schedule(), C.byref(v)))
        assert v.value == want, (set_v, v.value)
    ref = oracle.spmv(rp, cl, vl, x) if dtype == np.float64 else out[8192]
    for k in VC + vc4 + PLAIN:
        np.testing.assert_array_equal(out[k], ref, err_msg=f"variant {k}")


def test_value_codes_refused_past_255_values(queue, oracle):
    rp, cl, vl = quantized_banded(20_011, 2000)
    assert len(np.unique(vl)) > 255
    A = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    assert n_codes(A) == 0
    with pytest.raises(CgxError, match="value codes"):
        check(lib().cgx_csr_set_variant(A.schedule(), 34816))
    # plain SELL-P still works
    x = np.random.default_rng(1).standard_normal(len(rp) - 1)
    np.testing.assert_array_equal(spmv_all(queue, A, x, [8192])[8192],
                                  oracle.spmv(rp, cl, vl, x))


def test_value_codes_disabled_by_env(queue, oracle, monkeypatch):
    monkeypatch.setenv("CGX_VALUE_CODES", "0")
    rp, cl, vl = oracle.poisson(2, 40, 40, 1)
    A = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    assert n_codes(A) == 0


def test_value_codes_signed_zero_and_nonfinite(queue, oracle):
    # -0.0 and +0.0 are distinct dictionary entries (bit patterns); a stored
    # 0 times an Inf in x is NaN as in the reference, an empty slot is not
    rp, cl, vl = oracle.poisson(2, 16, 12, 1)
    vl = vl.copy()
    vl[3] = -0.0
    vl[10] = 0.0
    vl[11] = np.nan
    n = len(rp) - 1
    x = np.random.default_rng(7).standard_normal(n)
    x[5] = np.inf
    x[40] = -0.0
    A = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    assert n_codes(A) == 5
    y = spmv_all(queue, A, x, VC + VC4)
    ref = oracle.spmv(rp, cl, vl, x)
    for k in VC + VC4:
        np.testing.assert_array_equal(np.isnan(y[k]), np.isnan(ref))
        ok = ~np.isnan(ref)
        np.testing.assert_array_equal(y[k][ok], ref[ok])
        np.testing.assert_array_equal(np.signbit(y[k][ok]), np.signbit(ref[ok]))


@pytest.mark.parametrize("dim,n", [(2, 64), (3, 24)])
def test_cg_with_value_codes_matches_plain(oracle, monkeypatch, dim, n):
    """CG through the default path (autotune may pick value codes; small
    matrices take them by the size rule) equals the run with codes disabled
    bit for bit, and the oracle within the SURVEY §8(c) tolerances."""
    rp, cl, vl = oracle.poisson(dim, n, n, n)
    b = np.arange(1, len(rp), dtype=np.float64)
    xs = {}
    for vc in ("1", "0"):
        monkeypatch.setenv("CGX_VALUE_CODES", vc)
        cg = cga.CG.createCG()
        cg.setMatrix(vl, cl, rp)
        cg.setTarget(b)
        cg.solve(1e-8)
        v = C.c_int()
        check(lib().cgx_csr_variant(cg.A.schedule(), C.byref(v)))
        assert bool(v.value & 32768) == (vc == "1")
        xs[vc] = (cg.extract(), cg.iterations)
    np.testing.assert_array_equal(xs["1"][0], xs["0"][0])
    assert xs["1"][1] == xs["0"][1]
    xr, res = oracle.cg_solve(rp, cl, vl, b, 1e-8)
    assert abs(xs["1"][1] - res.iterations) <= 2
    assert rel(xs["1"][0], xr) <= 1e-10


@pytest.mark.parametrize("dim,n", [(2, 100), (3, 27)])
def test_cg_every_value_code_form_in_the_loop(oracle, monkeypatch, dim, n):
    """Every value-code form forced into the CG loop (k_cg_init and the
    fused k_spmv_dot, whose p.Ap takes the center pair from the gather in the
    lane-shift form) gives the plain SELL-P run's x and iteration count bit
    for bit; ragged sizes leave partial last slices."""
    rp, cl, vl = oracle.poisson(dim, n, n + 1, n - 2 if dim == 3 else 1)
    b = np.arange(1, len(rp), dtype=np.float64)
    out = {}
    for v in [8194] + VC + VC4:
        monkeypatch.setenv("CGX_SPMV_VARIANT", str(v))
        cg = cga.CG.createCG()
        cg.setMatrix(vl, cl, rp)
        cg.setTarget(b)
        cg.solve(1e-10)
        out[v] = (cg.extract(), cg.iterations)
    for v in VC + VC4:
        np.testing.assert_array_equal(out[v][0], out[8194][0], err_msg=f"variant {v}")
        assert out[v][1] == out[8194][1], v


# value-code templates (variant bit 8388608): the pipelined 4-bit forms
# (plain, stencil and plane march; default / non-temporal loads) with the
# slices whose code chunk equals a stored template reading it from LDS
VT = [9209856, 9209858, 10258432, 10258434, 12355584, 12355586]


def templates(m):
    nt, sl = C.c_int(), C.c_int64()
    check(lib().cgx_csr_templates(m.schedule(), C.byref(nt), C.byref(sl)))
    return nt.value, sl.value


def stream_bytes(m):
    b = C.c_int64()
    check(lib().cgx_csr_stream_bytes(m.schedule(), C.byref(b)))
    return b.value


@pytest.mark.parametrize("case", ["p3d_64", "p2d_512x256", "p3d_128x96x40"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_value_code_templates_bitexact(queue, oracle, case, dtype):
    """A slice reads its code chunk from a template only when the two are
    equal byte for byte (checked on the device at build), so Ap is
    bit-identical to the streamed-code forms and to the oracle; the stream
    shrinks by the template slices' chunks."""
    rp, cl, vl = {"p3d_64": lambda: oracle.poisson(3, 64, 64, 64),
                  "p2d_512x256": lambda: oracle.poisson(2, 512, 256, 1),
                  "p3d_128x96x40": lambda: oracle.poisson(3, 128, 96, 40)}[case]()
    n = len(rp) - 1
    A = Matrix(queue, vl, cl, rp, dtype=dtype)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    nt, nsl_t = templates(A)
    nsl = (n + 127) // 128
    assert 1 <= nt <= 8 and 64 <= nsl_t <= nsl, (nt, nsl_t, nsl)
    x = np.random.default_rng(11).standard_normal(n)
    x[[3, n // 2]] = [np.inf, -0.0]
    base = [821250, 1869826]
    out = spmv_all(queue, A, x, base + VT, dtype)
    ref = oracle.spmv(rp, cl, vl, x) if dtype == np.float64 else out[821250]
    for k in base + VT:
        np.testing.assert_array_equal(out[k], ref, err_msg=f"variant {k}")
    check(lib().cgx_csr_set_variant(A.schedule(), 1869826))
    b0 = stream_bytes(A)
    check(lib().cgx_csr_set_variant(A.schedule(), 10258434))
    v = C.c_int()
    check(lib().cgx_csr_variant(A.schedule(), C.byref(v)))
    assert v.value == 10264578
    assert stream_bytes(A) == b0 - 512 * nsl_t + 512 * nt


def test_value_code_templates_refused_without_them(queue, oracle, monkeypatch):
    monkeypatch.setenv("CGX_VT", "0")
    rp, cl, vl = oracle.poisson(3, 32, 32, 32)
    A = Matrix(queue, vl, cl, rp)
    check(lib().cgx_csr_set_sell(A.schedule(), 3))
    assert templates(A) == (0, 0)
    with pytest.raises(CgxError, match="templates"):
        check(lib().cgx_csr_set_variant(A.schedule(), VT[0]))


@pytest.mark.parametrize("mode", [1, 3, 4])
def test_value_code_templates_in_the_solver(oracle, monkeypatch, mode):
    """CG with the template form equals CG with streamed codes bit for bit
    (modes 1, 3 and 4), and the oracle to the §8(c) tolerances."""
    # x lines of 64 rows: a slice is two of them, so the interior slices of
    # every plane share one chunk (a template)
    rp, cl, vl = oracle.poisson(3, 64, 64, 48)
    b = np.arange(1, len(rp), dtype=np.float64)
    xs = {}
    for v in (1869826, 10258434):
        monkeypatch.setenv("CGX_SPMV_VARIANT", str(v))
        cg = cga.CG.createCG()
        cg.mode = mode
        cg.setMatrix(vl, cl, rp)
        cg.setTarget(b)
        cg.solve(1e-3)  # ||b|| = 4e7: 2e-11 relative (1e-8 sits at fp64's floor)
        xs[v] = (cg.extract(), cg.iterations)
    np.testing.assert_array_equal(xs[10258434][0], xs[1869826][0])
    assert xs[10258434][1] == xs[1869826][1]
    xr, res = oracle.cg_solve(rp, cl, vl, b, 1e-3)
    assert abs(xs[1869826][1] - res.iterations) <= 2
    assert rel(xs[10258434][0], xr) <= 1e-10
