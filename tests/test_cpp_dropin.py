"""The C++ drop-in boundary: include/CG.hpp & co. compile with the reference's
own driver (test/Tester.cpp, unmodified) and with our example, and run on the
GPU through libcgx.

CPU tests compile (g++ and clang++) and check that without a device the
program fails loudly. GPU tests run the binaries built by
`make -C examples [dropin]` and compare against the oracle's golden outputs.
"""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIBD = os.path.join(ROOT, "conjugategradient_amd")
REF_TEST = "/root/reference/test"
GOLD = os.path.join(ROOT, "tests", "golden")
TESTER = os.path.join(ROOT, "build", "dropin", "tester")
TESTER_CGXREAD = os.path.join(ROOT, "build", "dropin", "tester_cgxread")
EXAMPLE = os.path.join(ROOT, "build", "examples", "solve_poisson")


def _compile(cxx, srcs, out, extra=()):
    cmd = [cxx, "-std=c++17", "-O1", "-I" + INC, *extra, *srcs, "-o", out, "-L" + LIBD, "-lcgx",
           "-Wl,-rpath," + LIBD]
    return subprocess.run(cmd, capture_output=True, text=True)


@pytest.mark.parametrize("cxx", ["g++", "/opt/rocm/lib/llvm/bin/clang++"])
def test_reference_tester_compiles_unmodified(cxx, tmp_path):
    if not os.path.isdir(REF_TEST):
        pytest.skip("reference sources not present (GPU box)")
    if not shutil.which(cxx) and not os.path.exists(cxx):
        pytest.skip(f"{cxx} missing")
    out = str(tmp_path / "tester")
    r = _compile(cxx, [os.path.join(REF_TEST, "Tester.cpp"), os.path.join(REF_TEST, "mm_reader.cpp")],
                 out, ["-I" + REF_TEST])
    assert r.returncode == 0, r.stderr
    # no GPU here: the program must fail loudly, not fall back
    if not os.path.exists("/dev/kfd"):
        p = subprocess.run([out, os.path.join(GOLD, "poisson2d_16.mtx")], capture_output=True,
                           text=True)
        assert p.returncode != 0 and "cgx_create" in p.stderr


def test_reference_tester_compiles_with_cgx_loader(tmp_path):
    """Tester.cpp with examples/cgx_read_file.cpp in place of mm_reader.cpp."""
    if not os.path.isdir(REF_TEST):
        pytest.skip("reference sources not present (GPU box)")
    out = str(tmp_path / "tester_cgxread")
    r = _compile("g++", [os.path.join(REF_TEST, "Tester.cpp"),
                         os.path.join(ROOT, "examples", "cgx_read_file.cpp")], out,
                 ["-I" + REF_TEST])
    assert r.returncode == 0, r.stderr
    if not os.path.exists("/dev/kfd"):
        # the loader runs on the host before the queue fails for lack of a device
        p = subprocess.run([out, os.path.join(GOLD, "poisson2d_16.mtx")], capture_output=True,
                           text=True)
        assert p.returncode != 0 and "cgx_create" in p.stderr
        p = subprocess.run([out, str(tmp_path / "missing.mtx")], capture_output=True, text=True)
        assert p.returncode != 0 and "cannot open" in p.stderr


def test_example_compiles(tmp_path):
    out = str(tmp_path / "solve_poisson")
    r = _compile("g++", [os.path.join(ROOT, "examples", "solve_poisson.cpp")], out,
                 ["-Wall", "-Werror"])
    assert r.returncode == 0, r.stderr


def _parse(stdout):
    line = [ln for ln in stdout.splitlines() if re.match(r"^\d+ \d+ ", ln)][-1].split()
    return int(line[0]), int(line[1]), float(line[2]), float(line[3])


@pytest.mark.gpu
@pytest.mark.parametrize("exe", [TESTER, TESTER_CGXREAD], ids=["mm_reader", "cgx_loader"])
@pytest.mark.parametrize("name", ["poisson2d_16", "poisson2d_128", "poisson3d_16"])
def test_reference_tester_runs_on_gpu(name, exe):
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built (needs the reference sources at build time)")
    # bytes, decoded without newline translation: the progress line's "\r"
    # must survive (text=True would turn it into "\n")
    p = subprocess.run([exe, os.path.join(GOLD, name + ".mtx")], capture_output=True,
                       timeout=120)
    stdout, stderr = p.stdout.decode(), p.stderr.decode()
    assert p.returncode == 0, stderr[-2000:]
    n, nnz, ms, acc = _parse(stdout)
    g = np.load(os.path.join(GOLD, f"loader_{name}.npz"))
    assert n == len(g["rowptr"]) - 1 and nnz == len(g["val"])
    # Tester.cpp solves to 1e-24; accuracy() = ||b-Ax||^2/||x||^2 (Q6)
    gold = np.load(os.path.join(GOLD, f"cg_{name}.npz"))
    assert acc < 1e-24 and acc < 100 * float(gold["accuracy_1e-24"])
    _check_verbose_trace(stderr, n, int(gold["iters_1e-24"]))


# The std::clog sequence a Debuglevel::Verbose solver prints for Tester.cpp's
# calls (createCG, setMatrix, setTarget, solve, extract, getDimension,
# accuracy), in the reference's order and text:
REF_TRACE_HEAD = [
    r"Constructing CG Object",        # CG.hpp:63-64
    r"Setting Matrix",                # CG.hpp:89-90
    r"Solving System",                # CG.hpp:257-258
    r"work group size is \d+",        # VectorOperations.hpp:484-485 (vecops, CG.hpp:260)
    r"x init empty",                  # CG.hpp:292-295
    r"Prepared Memory",               # CG.hpp:306-308
    r"Init done",                     # CG.hpp:337-339
    r"Entering Loop",                 # CG.hpp:356-358
]
REF_TRACE_TAIL = [r"Finished solving", r"Calculating accuracy"]  # CG.hpp:450-453, :465-466


def _check_verbose_trace(stderr, n, oracle_bodies):
    lines = [ln for ln in stderr.split("\n") if "amdgpu.ids" not in ln]
    while lines and lines[-1] == "":
        lines.pop()
    head, prog, tail = lines[:len(REF_TRACE_HEAD)], lines[len(REF_TRACE_HEAD)], \
        lines[len(REF_TRACE_HEAD) + 1:]
    assert len(head) == len(REF_TRACE_HEAD) and all(
        re.fullmatch(w, h) for w, h in zip(REF_TRACE_HEAD, head)), lines
    assert tail == REF_TRACE_TAIL, lines
    # CG.hpp:428-434: "\r\033[2K" then (counter / N) * 100 and "%" after every
    # body whose counter is a multiple of 100 (default ostream format: %g);
    # the loop's std::endl (:451) ends the line
    steps = prog.split("\r\033[2K")
    assert steps[0] == "" and len(steps) >= 2, repr(prog)
    want = [f"{(100.0 * k / n) * 100:g}%" for k in range(len(steps) - 1)]
    assert steps[1:] == want, (steps[1:], want)
    # one line per started hundred bodies; the body count at 1e-24 follows
    # the summation order (report only), so a band
    assert abs(100 * (len(steps) - 1) - oracle_bodies) <= 100 + 0.1 * oracle_bodies


@pytest.mark.gpu
def test_example_runs_on_gpu(oracle):
    exe = EXAMPLE
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], check=True)
    p = subprocess.run([exe, "3", "16", "1e-8"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    n, nnz, ms, acc = _parse(p.stdout)
    assert n == 4096 and nnz == 27136
    it = int(re.search(r"iterations=(\d+)", p.stdout).group(1))
    assert abs(it - 76) <= 2  # 16^3 at 1e-8 -> 76 bodies
    assert acc < 1e-20
