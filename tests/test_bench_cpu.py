"""bench.py's host logic (no GPU): argument handling, the N-rank launcher,
and the byte accounting behind `value`, `roofline` and `csr_equivalent_GBs`."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_defaults_are_strong_scaling_of_256():
    a = bench.parse([])
    assert a.gpus == 1 and a.workload == "p3d_256" and a.grid is None and not a.weak
    assert a.transport == "auto"
    assert bench.parse(["--weak"]).weak


def test_launcher_starts_n_ranks(monkeypatch):
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    argv = ["--gpus", "4", "--steps", "9", "--grid", "512"]
    assert bench.main(argv) == 7  # the child's exit code is the parent's
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[cmd.index(os.path.join(ROOT, "bench.py")) + 1:] == argv
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.maybe_launch(bench.parse([]), []) is None


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="must match"):
        bench.maybe_launch(bench.parse(["--gpus", "4"]), ["--gpus", "4"])
    assert bench.maybe_launch(bench.parse(["--gpus", "2"]), ["--gpus", "2"]) is None


def test_byte_accounting():
    n, nnz = 256 ** 3, 117_047_296
    assert bench.b_alg(n, nnz) == 2_813_853_700  # 2.8139 GB
    assert bench.csr_spmv_bytes(n, nnz) == 12 * nnz + 4 * (n + 1) + 16 * n
    # r update 24 n; x/p update 40 n (mode 1) or 34 n averaged (mode 3)
    assert bench.update_bytes_per_iter(n, 1) == 64 * n
    assert bench.update_bytes_per_iter(n, 3) == 58 * n
    # mode 4: the p update lives in the SpMV (r, p_{k-1} read, p_k, Ap
    # written: 32 n beside the matrix stream); r update 24 n, x flush 12 n
    assert bench.update_bytes_per_iter(n, 4) == 36 * n
    assert bench.spmv_bytes_per_iter(1000, n, 4) == 1000 + 32 * n
    assert bench.spmv_bytes_per_iter(1000, n, 3) == 1000 + 16 * n
    # per iteration: mode 4 moves 6 n less than mode 3 (68 n against 74 n)
    m3 = bench.spmv_bytes_per_iter(0, n, 3) + bench.update_bytes_per_iter(n, 3)
    m4 = bench.spmv_bytes_per_iter(0, n, 4) + bench.update_bytes_per_iter(n, 4)
    assert (m3, m4) == (74 * n, 68 * n)


def test_job_cores_reports_host():
    info = bench.job_cores()
    assert 1 <= info["use"] <= info["affinity"] <= (os.cpu_count() or info["affinity"])
    assert "model" in info and info["nproc"] == os.cpu_count()


def test_pmc_csv_parsing():
    """roofline.traffic: per-kernel (2 FETCH_SIZE + WRITE_SIZE) KB x 1024 from
    rocprofv3 counter_collection.csv rows (the gfx950 FETCH correction)."""
    import io
    hdr = '"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n'
    fetch = io.StringIO(hdr +
                        '1,"void cgx::k_spmv_dot<double, 1875970>(cgx::CsrArgs, double const*)",'
                        '"FETCH_SIZE",100.0\n'
                        '2,"void cgx::k_spmv_dot<double, 1875970>(cgx::CsrArgs, double const*)",'
                        '"FETCH_SIZE",300.0\n'
                        '3,"void cgx::(anonymous namespace)::k_poisson<double>(int)","FETCH_SIZE",7\n')
    write = io.StringIO(hdr +
                        '1,"void cgx::k_spmv_dot<double, 1875970>(cgx::CsrArgs, double const*)",'
                        '"WRITE_SIZE",50.0\n')
    sums = {}
    bench.pmc_accumulate(fetch, "FETCH_SIZE", sums)
    bench.pmc_accumulate(write, "WRITE_SIZE", sums)
    out = bench.pmc_bytes(sums)
    assert out == {"k_spmv_dot<double, 1875970>": (2 * 200 + 50) * 1024}
    assert bench.kernel_base_name(
        "void cgx::(anonymous namespace)::k_poisson<double>(int, int)") == "k_poisson<double>"


def test_workload_choices():
    for w in ("p3d_256", "p3d_512", "p2d_4096", "p2d_128", "g3_standin"):
        assert bench.parse(["--workload", w]).workload == w
    assert bench.parse([]).workload == "p3d_256" and bench.parse([]).grid is None
