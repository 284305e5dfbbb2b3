"""libcgx's Matrix-Market loader and emitter (cgx_mm_read / cgx_mm_write_lower)
against the oracle's restatement of test/mm_reader.cpp read_file, the golden
loader fixtures (outputs of the reference loader built from its sources, see
tests/golden/make_golden.py) and the quirks Q1-Q3 of SURVEY §8. Host code
only: runs without a GPU.
"""
import glob
import os

import numpy as np
import pytest

import conjugategradient_amd as cga
from conjugategradient_amd._native import CgxError
from tests.util import irregular_spd

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _same(got, want_rp, want_cl, want_vl):
    data, cols, rows = got
    np.testing.assert_array_equal(rows, want_rp)
    np.testing.assert_array_equal(cols, want_cl)
    np.testing.assert_array_equal(data.view(np.uint64), np.asarray(want_vl).view(np.uint64))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "*.mtx"))))
@pytest.mark.parametrize("threads", [1, 4])
def test_read_file_matches_reference_golden(path, threads):
    name = os.path.splitext(os.path.basename(path))[0]
    g = np.load(os.path.join(GOLD, f"loader_{name}.npz"))
    _same(cga.read_file(path, threads), g["rowptr"], g["col"], g["val"])


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_quirks_inline(tmp_path, oracle):
    head = "%%MatrixMarket matrix coordinate real symmetric\n"
    cases = {
        # Q1: no comment line -> the size line is discarded, the first entry
        # becomes the size line
        "nocomment": head + "3 3 4\n1 1 4.0\n2 1 -1.0\n2 2 4.0\n3 3 4.0\n",
        # Q2: `general` is mirrored all the same
        "general": "%%MatrixMarket matrix coordinate real general\n% c\n3 3 3\n"
                   "1 1 2.0\n3 1 -1.5\n3 3 2.0\n",
        # Q3: row 2 (1-based) has no entry -> it vanishes from rowptr
        "emptyrow": head + "% c\n4 4 3\n1 1 1.0\n3 3 1.0\n4 4 1.0\n",
        # CRLF line ends, '+' signs, exponents, several comment lines
        "crlf": head.replace("\n", "\r\n") + "% a\r\n% b\r\n% c\r\n2 2 3\r\n"
                "+1 1 +4e0\r\n2 1 -1.25E-1\r\n2 2 4.\r\n",
        # malformed tail: the body ends at the first token that does not parse
        "badtail": head + "% c\n3 3 4\n1 1 4.0\n2 2 4.0\nxx 3 1.0\n3 3 4.0\n",
        # duplicates keep file order (originals before mirrors)
        "dups": head + "% c\n2 2 4\n2 1 1.0\n2 1 2.0\n1 1 3.0\n2 2 4.0\n",
        # entries not sorted in the file
        "unsorted": head + "% c\n3 3 5\n3 3 9.0\n2 1 1.0\n1 1 3.0\n3 2 7.0\n2 2 4.0\n",
    }
    for name, text in cases.items():
        p = _write(tmp_path, name + ".mtx", text)
        rp, cl, vl = oracle.read_mtx(p)
        for t in (1, 3):
            _same(cga.read_file(p, t), rp, cl, vl)
        if oracle.ref_available() and name != "dups":  # dups: order unspecified there
            rrp, rcl, rvl = oracle.ref_read_mtx(p)
            _same(cga.read_file(p), rrp, rcl, rvl)
    # Q1 / Q3 outcomes spelled out
    d, c, r = cga.read_file(str(tmp_path / "nocomment.mtx"))
    assert len(d) == 4      # 2 1 -1.0 mirrored + two diagonals; 1 1 4.0 was eaten
    d, c, r = cga.read_file(str(tmp_path / "emptyrow.mtx"))
    assert len(r) - 1 == 3 and list(c) == [0, 2, 3]


@pytest.mark.parametrize("kind", ["poisson3d", "irregular"])
def test_parallel_parse_large_and_round_trip(tmp_path, oracle, kind):
    if kind == "poisson3d":
        rp, cl, vl = oracle.poisson(3, 30, 28, 26)
    else:
        rp, cl, vl = irregular_spd(60_000, seed=11)
    p = str(tmp_path / f"{kind}.mtx")
    cga.write_mtx_lower(p, rp, cl, vl, threads=4)
    assert os.path.getsize(p) > 4 << 16          # several 64 KiB chunks
    orp, ocl, ovl = oracle.read_mtx(p)
    _same((ovl, ocl, orp), rp, cl, vl)            # the emitter round-trips exactly
    for t in (1, 2, 7, 16):
        _same(cga.read_file(p, t), rp, cl, vl)
    # the oracle's emitter output reads identically too
    q = str(tmp_path / f"{kind}_oracle.mtx")
    oracle.write_mtx_lower(q, rp, cl, vl)
    _same(cga.read_file(q), rp, cl, vl)


def test_misaligned_chunks_fall_back_to_sequential(tmp_path, oracle):
    # triplets wrapped over lines: chunk boundaries at line starts split
    # triplets, so the parser must notice and parse sequentially
    rp, cl, vl = oracle.poisson(2, 60, 60, 1)
    lines = ["%%MatrixMarket matrix coordinate real symmetric", "% wrapped", "3600 3600 0"]
    n = len(rp) - 1
    for i in range(n):
        for k in range(rp[i], rp[i + 1]):
            if cl[k] <= i:
                lines.append(f"{i + 1} {cl[k] + 1}")
                lines.append(repr(float(vl[k])))
    p = _write(tmp_path, "wrapped.mtx", "\n".join(lines) + "\n")
    orp, ocl, ovl = oracle.read_mtx(p)
    for t in (1, 8):
        _same(cga.read_file(p, t), orp, ocl, ovl)


def test_errors(tmp_path):
    with pytest.raises(CgxError, match="cannot open"):
        cga.read_file(str(tmp_path / "missing.mtx"))
    p = _write(tmp_path, "banner.mtx", "%%MatrixMarket matrix coordinate\n% c\n1 1 1\n1 1 1.0\n")
    with pytest.raises(CgxError, match="5 words"):
        cga.read_file(p)
    p = _write(tmp_path, "size.mtx",
               "%%MatrixMarket matrix coordinate real symmetric\n% c\n1 1\n1 1 1.0\n")
    with pytest.raises(CgxError, match="size line"):
        cga.read_file(p)
    p = _write(tmp_path, "zero.mtx",
               "%%MatrixMarket matrix coordinate real symmetric\n% c\n2 2 1\n0 1 1.0\n")
    with pytest.raises(CgxError, match="index < 1"):
        cga.read_file(p)
    p = _write(tmp_path, "empty.mtx",
               "%%MatrixMarket matrix coordinate real symmetric\n% c\n2 2 0\n")
    with pytest.raises(CgxError, match="no entries"):
        cga.read_file(p)
