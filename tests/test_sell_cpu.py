"""SELL-64 layout (cgx_sell_plan, host-only) checked on the CPU.

The test emulates spmv_sell's addressing (cgx_kernels.hip) lane by lane in
numpy. Every index the kernel forms must fall inside the arrays
cgx_csr_create allocates:
  * values: value_slots + 8 * 64, for the chunk of slack;
  * index words: nidx;
  * dictionary pool: ndict;
  * gathered x: n.
Both layouts are covered: 1 and 2 rows per lane. With values packed the
way k_sell_pack packs them, the emulated row sums
must equal the oracle's SpMV bit for bit.
"""
import ctypes as C

import numpy as np
import pytest

from conjugategradient_amd._native import check, lib
from tests.util import irregular_spd

ROWS = 64
PAD = 0xFF


def sell_plan(rp, cl, R=1):
    L = lib()
    nsl, ndict, nidx, slots = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
    sl = C.POINTER(C.c_int64)()
    dic = C.POINTER(C.c_int32)()
    idx = C.POINTER(C.c_uint64)()
    rp = np.ascontiguousarray(rp, np.int32)
    cl = np.ascontiguousarray(cl, np.int32)
    check(L.cgx_sell_plan(rp.ctypes.data, cl.ctypes.data, len(rp) - 1, R, C.byref(nsl), C.byref(sl),
                          C.byref(ndict), C.byref(dic), C.byref(nidx), C.byref(idx),
                          C.byref(slots)))
    if nsl.value == 0:
        return None
    out = (np.ctypeslib.as_array(sl, shape=(nsl.value, 4)).copy(),
           np.ctypeslib.as_array(dic, shape=(ndict.value,)).copy(),
           np.ctypeslib.as_array(idx, shape=(max(nidx.value, 1),))[:nidx.value].copy(),
           slots.value)
    for p in (sl, dic, idx):
        L.cgx_free_host(C.cast(p, C.c_void_p))
    return out


def pack_values(rp, vl, sl, slots, R=1):
    """k_sell_pack: slot j of row i = val[rowptr[i] + j], 0 past the row."""
    n = len(rp) - 1
    sval = np.zeros(slots + 8 * ROWS * R, vl.dtype)
    H = ROWS * R
    for q, (voff, _, _, w) in enumerate(sl):
        for li in range(H):
            i = q * H + li
            if i >= n:
                continue
            l, r = divmod(li, R)
            a, e = rp[i], rp[i + 1]
            for j in range(e - a):
                sval[voff + (j * ROWS + l) * R + r] = vl[a + j]
    return sval


def emulate_spmv(rp, sl, dic, idx, sval, x, R=1):
    """spmv_sell (R = 1) / sell_slice2 (R = 2), with every index the kernel
    forms checked against the array extents cgx_csr_create allocates."""
    n = len(rp) - 1
    y = np.zeros(n)
    lane = np.arange(ROWS)
    H = ROWS * R
    if R == 2:   # 16-byte loads: voff / ioff must be even (aligned)
        assert (sl[:, 0] % 2 == 0).all() and (sl[:, 1] % 2 == 0).all()
    for q, (voff, ioff, dbase, w) in enumerate(sl):
        assert dbase + ROWS <= len(dic)
        dv = dic[dbase + lane]
        for r in range(R):
            row = q * H + R * lane + r
            live = row < n
            rowc = np.where(live, row, n - 1)
            acc = np.zeros(ROWS)
            for c in range(0, w, 8):
                wi = ioff + ((c >> 3) * ROWS + lane) * R + r
                assert wi.max() < len(idx)
                iw = idx[wi]
                for j in range(8):
                    vi = voff + ((c + min(j, w - 1 - c)) * ROWS + lane) * R + r
                    assert vi.max() < len(sval)
                    v = sval[vi]
                    k = ((iw >> np.uint64(8 * j)) & np.uint64(0xFF)).astype(np.int64)
                    off = dv[(k * 4 // 4) % ROWS]              # ds_bpermute
                    g_idx = np.where(k != PAD, row + off, rowc)
                    assert g_idx.min() >= 0 and g_idx.max() < n
                    g = x[g_idx]
                    with np.errstate(invalid="ignore"):
                        t = acc + v * g
                    acc = np.where(k != PAD, t, acc)
            y[row[live]] = acc[live]
    return y


def cases(oracle):
    from tests.test_gpu_sell import banded
    return {
        "poisson3d_ragged": oracle.poisson(3, 23, 19, 17),
        "poisson2d": oracle.poisson(2, 40, 33, 1),
        "banded": banded(5_003, half=9),
        "empty_rows": banded(2_001, half=6, empty_every=13),
        "tiny": (np.array([0, 1, 3, 4], np.int32), np.array([0, 0, 1, 2], np.int32),
                 np.array([2.0, -1.0, 3.0, 4.0])),
        "wide": banded(777, half=25),   # rows > 8 entries: several index words
        "mid": banded(901, half=12),    # 25 offsets: SELL-P with u32 masks
    }


@pytest.mark.parametrize("R", [1, 2])
@pytest.mark.parametrize("case", ["poisson3d_ragged", "poisson2d", "banded", "empty_rows",
                                  "tiny", "wide"])
def test_sell_layout_in_bounds_and_bitexact(oracle, case, R):
    rp, cl, vl = cases(oracle)[case]
    plan = sell_plan(rp, cl, R)
    assert plan is not None, case
    sl, dic, idx, slots = plan
    n = len(rp) - 1
    assert len(sl) == (n + ROWS * R - 1) // (ROWS * R)
    assert (sl[:, 3] <= 64).all() and slots == (sl[:, 3] * ROWS * R).sum()
    # dictionary indices < 64, every real entry present exactly once
    b = idx.view(np.uint8)
    assert ((b == PAD) | (b < 64)).all()
    assert (b != PAD).sum() == len(vl)
    sval = pack_values(rp, vl, sl, slots, R)
    x = np.random.default_rng(1).standard_normal(n)
    np.testing.assert_array_equal(emulate_spmv(rp, sl, dic, idx, sval, x, R),
                                  oracle.spmv(rp, cl, vl, x))


def test_sell_dictionaries_are_shared(oracle):
    rp, cl, _ = oracle.poisson(3, 32, 32, 32)
    sl, dic, _, _ = sell_plan(rp, cl)
    # interior slices of a stencil share a handful of dictionaries
    assert len(np.unique(sl[:, 2])) < 40
    assert len(dic) < 40 * 7 + 64


def test_sell_rejects_scattered_and_long_rows():
    rp, cl, _ = irregular_spd(20_000, seed=4)
    assert sell_plan(rp, cl) is None and sell_plan(rp, cl, 2) is None
    rp, cl, _ = irregular_spd(5_000, seed=5, hub=3000)   # one row of ~3000 entries
    assert sell_plan(rp, cl) is None


# ---- SELL-P (pattern slots + row masks, 2 rows per lane) ------------------

def sellp_plan(rp, cl):
    L = lib()
    nsl, npat, slots, mw = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int()
    sl = C.POINTER(C.c_int64)()
    pat = C.POINTER(C.c_int32)()
    rp = np.ascontiguousarray(rp, np.int32)
    cl = np.ascontiguousarray(cl, np.int32)
    check(L.cgx_sellp_plan(rp.ctypes.data, cl.ctypes.data, len(rp) - 1, C.byref(nsl), C.byref(sl),
                           C.byref(npat), C.byref(pat), C.byref(slots), C.byref(mw)))
    if nsl.value == 0:
        return None
    out = (np.ctypeslib.as_array(sl, shape=(nsl.value, 4)).copy(),
           np.ctypeslib.as_array(pat, shape=(npat.value,)).copy(), slots.value, mw.value)
    for p in (sl, pat):
        L.cgx_free_host(C.cast(p, C.c_void_p))
    return out


def sellp_pack(rp, cl, vl, sl, pat, slots):
    """k_sellp_pack: entry of offset o goes to the slot of o in the slice's
    pattern; mask bit per set slot; rows past n: zeros, mask 0."""
    n = len(rp) - 1
    H = 2 * ROWS
    sval = np.zeros(slots + 8 * H, vl.dtype)
    mask = np.zeros(len(sl) * H, np.uint32)
    for q, (voff, _, base, w) in enumerate(sl):
        P = pat[base:base + w]
        for li in range(H):
            i = q * H + li
            if i >= n:
                continue
            l, r = divmod(li, 2)
            k, e = rp[i], rp[i + 1]
            bits = 0
            for j in range(w):
                if k < e and cl[k] - i == P[j]:
                    sval[voff + (j * ROWS + l) * 2 + r] = vl[k]
                    bits |= 1 << j
                    k += 1
            assert k == e, "every entry lands in a slot"
            mask[i] = bits
    return sval, mask


def sellp_emulate(rp, sl, pat, sval, mask, x):
    """sellp_slice2: pair loads at clamp(r0 + o, 0, nx - 2), halves selected."""
    n = len(rp) - 1
    nx = len(x)
    y = np.zeros(n)
    lane = np.arange(ROWS)
    for q, (voff, _, base, w) in enumerate(sl):
        r0 = q * 2 * ROWS + 2 * lane
        m0, m1 = mask[r0], mask[r0 + 1]
        acc0, acc1 = np.zeros(ROWS), np.zeros(ROWS)
        for c in range(0, w, 8):
            for j in range(8):
                jj = min(j, w - 1 - c)
                vi = voff // 2 + (c + jj) * ROWS + lane
                assert vi.max() * 2 + 1 < len(sval)
                v0, v1 = sval[2 * vi], sval[2 * vi + 1]
                assert base + min(c + j, w - 1) < len(pat)
                o = pat[base + min(c + j, w - 1)]
                b = r0 + o
                cb = np.clip(b, 0, nx - 2)
                g = np.stack([x[cb], x[cb + 1]])            # the pair load, in bounds
                g0 = np.where(b <= nx - 2, g[0], g[1])
                g1 = np.where(b >= 0, g[1], g[0])
                s = c + j
                if s < w:
                    on0 = (m0 >> s) & 1 == 1
                    on1 = (m1 >> s) & 1 == 1
                    with np.errstate(invalid="ignore"):
                        acc0 = np.where(on0, acc0 + v0 * g0, acc0)
                        acc1 = np.where(on1, acc1 + v1 * g1, acc1)
        for r, acc in ((0, acc0), (1, acc1)):
            rows = r0 + r
            live = rows < n
            y[rows[live]] = acc[live]
    return y


@pytest.mark.parametrize("case", ["poisson3d_ragged", "poisson2d", "banded", "empty_rows",
                                  "tiny", "mid"])
def test_sellp_layout_in_bounds_and_bitexact(oracle, case):
    rp, cl, vl = cases(oracle)[case]
    plan = sellp_plan(rp, cl)
    assert plan is not None, case
    sl, pat, slots, mw = plan
    n = len(rp) - 1
    assert len(sl) == (n + 2 * ROWS - 1) // (2 * ROWS)
    assert (sl[:, 3] <= 32).all() and mw == sl[:, 3].max()
    for (_, _, base, w) in sl:           # patterns sorted, strictly ascending
        P = pat[base:base + w]
        assert (np.diff(P) > 0).all()
    sval, mask = sellp_pack(rp, cl, vl, sl, pat, slots)
    x = np.random.default_rng(2).standard_normal(n)
    np.testing.assert_array_equal(sellp_emulate(rp, sl, pat, sval, mask, x),
                                  oracle.spmv(rp, cl, vl, x))


def test_sellp_rejects(oracle):
    # scattered columns, or a band of 51 offsets: patterns wider than 32
    rp, cl, _ = irregular_spd(20_000, seed=4)
    assert sellp_plan(rp, cl) is None
    rp, cl, _ = cases(oracle)["wide"]
    assert sellp_plan(rp, cl) is None
    # a row with unsorted columns
    rp = np.array([0, 2, 3], np.int32)
    cl = np.array([1, 0, 1], np.int32)
    assert sellp_plan(rp, cl) is None


def test_sellp_refuses_the_upper_ranks_remapped_slab(oracle):
    """Why a partitioned matrix's boundary slices are placeholders in its SELL
    copy (cgx_dist.cpp): a rank's local numbering puts its own
    rows first and its ghosts after them, so a row of rank 1 that gathers
    from the plane below lists that ghost (local n_local + k) first in its
    CSR order. The plain SELL-P plan refuses such a slab (its slots sum in
    ascending local offset order); rank 0's slab, whose ghosts lie above,
    and every row of rank 1 but its first plane's is sorted."""
    from conjugategradient_amd._native import check, lib
    L = lib()
    nx, nz = 128, 8
    rp, cl, _ = oracle.poisson(3, nx, nx, nz)
    n = len(rp) - 1
    nl = n // 2
    plane = nx * nx
    plans = []
    for rank in (0, 1):
        b = rank * nl
        r = (rp[b:b + nl + 1] - rp[b]).astype(np.int32)
        c = cl[rp[b]:rp[b + nl]].astype(np.int32).copy()
        begins = (C.c_int64 * 2)(0, nl)
        counts = (C.c_int64 * 2)(nl, nl)
        ng, gh, rc = C.c_int64(), C.POINTER(C.c_int64)(), (C.c_int64 * 2)()
        check(L.cgx_plan_ghosts(nl, b, len(c), c.ctypes.data, 2, begins, counts, C.byref(ng),
                                C.byref(gh), rc))
        assert ng.value == plane
        check(L.cgx_plan_remap(nl, b, len(c), c.ctypes.data, ng.value, gh))
        L.cgx_free_host(gh)
        plans.append((r, c))
    (r0, c0), (r1, c1) = plans
    assert sellp_plan(r0, c0) is not None
    assert sellp_plan(r1, c1) is None
    # exactly its first plane's rows are the unsorted ones
    unsorted = [i for i in range(nl) if (np.diff(c1[r1[i]:r1[i + 1]]) <= 0).any()]
    assert unsorted == list(range(plane))
