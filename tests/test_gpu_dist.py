"""Multi-rank device path (cgx_dist.cpp) on the GPU box.

RCCL refuses two ranks on one GPU, so on a single-GPU box the multi-rank
runs use the host-staged transport (cgx_dist_init_host over gloo): the same
halo plan, ghost area, pack kernel, all-reduce points and stop rule as the
RCCL path, only the bytes travel through host memory. "host-peer" runs add
the device peer transport (cgx_peer.hip) on top: the ranks (processes) map
each other's mailboxes and landing buffers with hipIpc on the shared GPU and
run the iteration's halo exchange and all-reduces as kernels, exactly as on
an 8-GPU node (where the stores cross xGMI instead). The RCCL transport
itself runs at world size 1 here and at 1/2/4/8 in the driver's scaling
bench (bench.py). Each run is a tests/dist_check.py job under
torch.distributed.run; rank 0 compares x with the oracle (rel 1e-10,
bodies +-2)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, transport, grid, mode=0, extra=(), timeout=300, env=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_check.py"), "--transport", transport,
           "--grid", str(grid), "--mode", str(mode), *extra]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT,
                       env=None if env is None else {**os.environ, **env})
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("nproc,transport,grid,mode", [(1, "rccl", 32, 0), (2, "host", 24, 0),
                                                       (3, "host", 20, 0), (2, "host", 20, 3),
                                                       (1, "rccl", 24, 3), (2, "host-peer", 24, 0),
                                                       (3, "host-peer", 20, 0),
                                                       (2, "host-peer", 20, 1),
                                                       (4, "host-peer", 16, 3)])
def test_partitioned_solve_matches_oracle(nproc, transport, grid, mode):
    r = _run(nproc, transport, grid, mode)
    assert r["ok"], r
    if nproc > 1:
        # slab partition of a 3-D grid: every rank has ghosts, inner ranks 2 nbrs
        assert all(g > 0 for g in r["ghosts"])
        assert r["neighbours"][0] == 1
        # the SELL copy is split: interior slices run while the halo travels
        assert all(ni > 0 and nb > 0 for ni, nb in r["split"]), r["split"]
    # the device peer transport (halo push / wait kernels, mailbox all-reduce
    # over hipIpc-mapped memory) passed its self-test on every rank and ran
    # the iteration, graph-captured
    assert r["peer"] == [int(transport.endswith("-peer"))] * nproc
    if transport.endswith("-peer") and nproc > 1:
        # every rank shares this one GPU: the one-waiter form runs
        assert r["peer_form"] == [[nproc, 1]] * nproc, r["peer_form"]


@pytest.mark.parametrize("nproc,transport", [(1, "rccl"), (2, "host-peer"), (4, "host-peer"),
                                             (8, "host-peer")])
def test_partitioned_x_independent_of_world_size(nproc, transport):
    """The dots are double-length sums (round 6) from the threads through the
    workgroup partials to the peer transport's world sum of the ranks' pairs
    in rank order, rounded once: x after 30 bodies is bit for bit the dd
    oracle's (oracle.cg_solve_dd) on 1 rank (RCCL at world size 1) and on 2,
    4 and 8 ranks, in mode 3 and in mode 4 (lean interior)."""
    for mode in (3, 4):
        if mode == 4 and nproc == 1:
            continue  # (the partitioned mode 4 needs the peer transport)
        r = _run(nproc, transport, 64, mode, ["--nxy", "128", "--bodies", "30"], env=LEAN)
        assert r["ok"], r
        assert r["bodies"] == 30 and r["mode_run"] == mode
        assert r["dd_equal"] is True, (nproc, mode, r["rel_err"])


@pytest.mark.parametrize("transport,mode", [("host", 0), ("host-peer", 3), ("host-async", 3)])
def test_eight_way_split(transport, mode):
    """Config 4's 8-way row split (BASELINE.json configs[3]) as 8 ranks on this
    one GPU: a 64^3 grid in 8-plane slabs, 6 inner ranks with two neighbours
    and 2 end ranks with one; 80 bodies at tol 0 against the oracle's
    iteration (rel 1e-10). (A 1e-8 solve of 64^3 with b_i = i + 1 stops at
    the rounding floor, ||b|| ~ 8e7, where the body count is noise.)"""
    r = _run(8, transport, 64, mode, ["--bodies", "80"])
    assert r["ok"], {k: r[k] for k in ("rel_err", "bodies", "oracle_bodies", "accuracy")}
    assert r["bodies"] == 80
    assert r["neighbours"] == [1, 2, 2, 2, 2, 2, 2, 1], r["neighbours"]
    assert r["ghosts"] == [64 * 64] + [2 * 64 * 64] * 6 + [64 * 64], r["ghosts"]
    assert all(ni > 0 and nb > 0 for ni, nb in r["split"]), r["split"]
    assert r["peer"] == [int(transport.endswith("-peer"))] * 8
    if transport == "host-peer":
        assert r["peer_form"] == [[8, 1]] * 8, r["peer_form"]
    if transport == "host-async":
        assert all(c >= 80 for c in r["async_exchanges"]), r["async_exchanges"]


@pytest.mark.parametrize("nproc,grid,mode", [(2, 24, 0), (3, 20, 3)])
def test_async_host_halo_matches_synchronous(nproc, grid, mode):
    """The overlapped halo ordering of the RCCL branch (cgx_dist.cpp
    dist_halo_post: pack, ev_pack, exchange on the comm stream, ev_halo; the
    solver stream runs the interior slices and waits on ev_halo before the
    boundary slices) exercised on one GPU: the host transport's exchange runs
    as a host function on the comm stream (cgx_dist_host_async). x must be
    bit-identical to the synchronous exchange and match the oracle."""
    ra = _run(nproc, "host-async", grid, mode)
    rs = _run(nproc, "host", grid, mode)
    assert ra["ok"] and rs["ok"], (ra, rs)
    assert all(ni > 0 and nb > 0 for ni, nb in ra["split"]), ra["split"]
    # every body of every rank posted its exchange on the comm stream
    assert all(c >= ra["bodies"] for c in ra["async_exchanges"]), ra
    assert rs["async_exchanges"] == [0] * nproc
    assert ra["bodies"] == rs["bodies"]
    assert ra["x_sha"] == rs["x_sha"]


@pytest.mark.parametrize("nproc,transport", [(2, "host-peer"), (2, "host"), (3, "host-peer")])
def test_partitioned_lean_interior(nproc, transport):
    """Every rank's slab gets the SELL-P value-code layout and the lean walk
    (DESIGN.md §9): the boundary rows (ghost columns; from a lower rank they
    are numbered after the own rows, so those rows are unsorted locally) are
    placeholders in the SELL copy and run as CSR-stream blocks in the
    boundary launch; the lean layout skips their slices (class 0xfe) and the
    interior launch walks the rest (with the halo push in its first
    workgroups on the peer transport). 128 x 128 x 48 over 2 and 3 ranks,
    the walk forced at creation; x against the oracle (rel 1e-10)."""
    r = _run(nproc, transport, 48, 3, ["--nxy", "128", "--bodies", "30"],
             env={"CGX_SPMV_VARIANT": "33554432:0"})
    assert r["ok"], r
    assert r["bodies"] == 30
    planes = 48 // nproc
    for var, lean_slices in r["variant_lean_slices"]:
        assert var & 33554432, r["variant_lean_slices"]
        # nearly every slice of the slab but its boundary plane(s) is lean
        # (a few interior slices keep the per-slice form)
        assert lean_slices >= (planes - 3) * 128, r["variant_lean_slices"]
    assert all(ni > 0 and nb > 0 for ni, nb in r["split"]), r["split"]


LEAN = {"CGX_SPMV_VARIANT": "33554432:0"}


@pytest.mark.parametrize("nproc", [2, 3, 4, 8])
def test_partitioned_mode4_bit_identical_to_mode3(nproc):
    """Mode 4 on the partitioned body (round 5): kernel 1 walks the interior
    forming p_k = r + beta p_{k-1} and pushes the formed p_k of the send rows
    from its first workgroups, kernel 2 runs the boundary rows after the
    neighbours' pushes, kernel 3 is update_r with the p.Ap all-reduce, the
    stop rule and the slot-3 x flush, its last workgroup all-reducing r.r.
    Its SpMV partials split as mode 3's (the walk's grid, the boundary row
    blocks' grid) and every formed value is mode 3's p update, so x is bit
    for bit mode 3's; 30 bodies at tol 0 against the oracle (rel 1e-10)."""
    args = ["--nxy", "128", "--bodies", "30"]
    grid = 64 if nproc == 8 else 48
    r4 = _run(nproc, "host-peer", grid, 4, args, env=LEAN)
    r3 = _run(nproc, "host-peer", grid, 3, args, env=LEAN)
    assert r4["ok"] and r3["ok"], (r4, r3)
    assert r4["mode_run"] == 4 and r3["mode_run"] == 3
    assert r4["bodies"] == r3["bodies"] == 30
    for var, _ in r4["variant_lean_slices"]:
        assert var & 33554432, r4["variant_lean_slices"]
    assert r4["x_sha"] == r3["x_sha"], (r4, r3)
    if nproc > 2:  # inner ranks: two neighbours, two pushes and two waits per body
        assert r4["neighbours"][1] == 2, r4["neighbours"]


@pytest.mark.parametrize("nproc", [2, 8])
def test_peer_forms_bit_identical(nproc):
    """The device peer transport's two iteration forms (cgx_dist_peer_form,
    DESIGN.md §9 "Ranks sharing a GPU"): the fused form waits inside the
    consuming kernels (every workgroup of the boundary launch polls the push
    flags, every workgroup of update_r and of the p update polls the dot
    mailboxes: the 8-GPU node's form), the one-waiter form puts one
    one-workgroup launch in front of each (k_peer_wait, k_peer_allreduce),
    which ranks sharing a GPU need. Both sum the same partials in the same
    order, so x is bit for bit the same, in mode 3 and in mode 4."""
    args = ["--nxy", "128", "--bodies", "30"]
    grid = 16 * nproc
    for mode in (3, 4):
        rf = _run(nproc, "host-peer", grid, mode, args, env={**LEAN, "CGX_PEER_ONE_WAITER": "0"})
        ro = _run(nproc, "host-peer", grid, mode, args, env=LEAN)
        assert rf["ok"] and ro["ok"], (rf, ro)
        assert rf["peer_form"] == [[nproc, 0]] * nproc, rf["peer_form"]
        assert ro["peer_form"] == [[nproc, 1]] * nproc, ro["peer_form"]
        assert rf["mode_run"] == ro["mode_run"] == mode
        assert rf["bodies"] == ro["bodies"] == 30
        assert rf["x_sha"] == ro["x_sha"], (mode, rf, ro)


@pytest.mark.parametrize("form", ["0", "1"])
def test_partitioned_mixed_modes_agree(form):
    """Auto mode decides per rank (each rank's own autotune), so ranks can run
    mode 3 and mode 4 side by side: both modes push, wait and
    all-reduce with the same tags per body (push / wait at the body's base,
    p.Ap at base + 1, r.r at base + 2, the stop rule on the starting r.r).
    Rank 0 in mode 3, rank 1 in mode 4, to tolerance: the same bodies and x
    bit for bit as both ranks in mode 3, in both peer forms."""
    args = ["--nxy", "128"]
    env = {**LEAN, "CGX_PEER_ONE_WAITER": form}
    rm = _run(2, "host-peer", 48, "3,4", args, env=env)
    r3 = _run(2, "host-peer", 48, 3, args, env=env)
    assert rm["ok"] and r3["ok"], (rm, r3)
    assert rm["modes_run"] == [3, 4] and r3["modes_run"] == [3, 3]
    assert rm["bodies"] == r3["bodies"]
    assert rm["x_sha"] == r3["x_sha"], (rm, r3)


def test_partitioned_mode4_stop_rule_and_resumed_runs():
    """The stop rule and the run boundaries of partitioned mode 4: solved to
    tolerance, and the same solve split into cgx_cg_run calls of 40 bodies
    (each run ends with its x flush; kernel 3's last workgroup has already
    recorded the world r.r the next run's kernel 1 forms beta from). Both
    end on the oracle's body count (+-2) and x (rel 1e-10), bit-identical to
    each other and to mode 3."""
    args = ["--nxy", "128"]
    r1 = _run(2, "host-peer", 48, 4, args, env=LEAN)
    rr = _run(2, "host-peer", 48, 4, args + ["--runs", "3"], env=LEAN)
    r3 = _run(2, "host-peer", 48, 3, args, env=LEAN)
    assert r1["ok"] and rr["ok"] and r3["ok"], (r1, rr, r3)
    assert r1["mode_run"] == rr["mode_run"] == 4
    assert r1["bodies"] == rr["bodies"] == r3["bodies"]
    assert r1["x_sha"] == rr["x_sha"] == r3["x_sha"], (r1, rr, r3)


def test_partitioned_ranks_share_the_sellp_layout():
    """Without forcing a form, the ranks above rank 0 (whose boundary rows
    gather ghosts numbered after their own rows) get the SELL-P value-code
    layout as rank 0 does, not the dictionary SELL fallback of an unsorted
    matrix (round 4 finding)."""
    r = _run(3, "host", 48, 3, ["--nxy", "128", "--bodies", "20"])
    assert r["ok"], r
    fams = {var & (2048 | 4096 | 8192 | 32768) for var, _ in r["variant_lean_slices"]}
    assert fams == {8192 | 32768}, r["variant_lean_slices"]


def test_partitioned_slab_of_the_8gpu_config():
    """BASELINE config 4's per-rank shape: 512^3 over 8 GPUs gives each rank a
    512 x 512 x 64 slab and 2 MiB halo planes. Two such slabs (global
    512 x 512 x 128, 33.5 M rows) on the host transport, 40 bodies at tol 0,
    against the oracle's OpenMP iteration (rel 1e-10)."""
    r = _run(2, "host", 128, 0, ["--nxy", "512", "--bodies", "40"], timeout=900)
    assert r["ok"], r
    assert r["bodies"] == 40 and r["grid"] == [512, 512, 128]
    assert r["ghosts"] == [512 * 512, 512 * 512]  # one plane from the other slab
    assert all(ni > 0 and nb > 0 for ni, nb in r["split"]), r["split"]


def test_bench_two_ranks_validates_peer_transport():
    """bench.py at N > 1 uses the device peer transport only after
    validate_peer solved a small slab problem over it and over the setup
    transport to the same answer (accuracy, bodies +-2, x to 1e-10). On the
    one-GPU box the setup transport is the host one (--transport host-peer);
    on an 8-GPU node it is RCCL (--transport auto)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--grid", "64",
           "--steps", "20", "--warmup", "5", "--transport", "host-peer", "--no-cpu",
           "--profile-steps", "0", "--master-port", str(_port())]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["steps"] == 20
    v = line["config"]["transport_validation"]
    assert v["ok"], v
    assert v["x_rel_peer_vs_setup"] <= 1e-10
    assert line["config"]["transport"].startswith("peer")
    # the RCCL iteration beside it: not on one GPU (RCCL refuses shared devices)
    assert "RCCL" in line["config"]["rccl_iteration"]["skipped"]


def test_bench_two_ranks_autotune_takes_the_lean_interior():
    """The metric's grid over two ranks (256 x 256 x 128 slabs, past the
    autotune's size rule): each rank's autotune times the SELL forms and the
    lean walk on its interior slices (the boundary slices are the boundary
    launch's) and takes the lean walk, which then carries the partitioned
    body (the lean candidate used to be timed as CSR-stream)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--grid", "256",
           "--steps", "20", "--warmup", "5", "--transport", "host-peer", "--no-cpu",
           "--profile-steps", "0", "--master-port", str(_port())]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = line["config"]
    assert cfg["spmv_variant"] & 33554432, cfg["spmv_variant"]
    hows = {f["how"] for f in cfg["spmv_autotune"]["forms"]}
    assert "lean walk (interior slices)" in hows and "k_spmv_dot (interior slices)" in hows, hows
    # a split matrix's SELL forms are timed on its interior slices only
    for f in cfg["spmv_autotune"]["forms"]:
        if f["variant"] & (2048 | 8192) and f["how"].startswith("k_spmv_dot"):
            assert f["how"] == "k_spmv_dot (interior slices)", f


def test_bench_four_ranks_auto_mode4_validated():
    """128^3 over 4 ranks (128 x 128 x 32 slabs, inside the auto rule's 4 M
    rows) with the lean interior on every rank: bench.py's auto mode takes the
    partitioned mode 4 only after every rank agreed and it solved a 128 x 128
    slab problem over the peer transport to the setup transport's answer
    (config.transport_validation.mode4), then times it. (256^3 over 4 ranks:
    test_bench_four_ranks_256_on_one_gpu.)"""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--grid", "128",
           "--steps", "20", "--warmup", "5", "--transport", "host-peer", "--no-cpu",
           "--profile-steps", "0", "--force-lean", "--master-port", str(_port())]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = line["config"]
    v4 = cfg["transport_validation"]["mode4"]
    assert v4["ok"] and v4["peer_mode"] == 4, v4
    assert cfg["iteration"].startswith("3 launches (interior walk forming p_k"), cfg["iteration"]
    assert cfg["peer_fallback_reason"] is None, cfg["peer_fallback_reason"]


def test_bench_four_ranks_256_on_one_gpu():
    """The metric's 256^3 grid over 4 ranks sharing this one GPU (256 x 256 x
    64 slabs, 4.2 M rows each), the lean interior forced: in round 5 every
    rank's warm-up timed out in mode 3 and in mode 4, because the boundary
    launches polled for pushes with their whole grids resident and held the
    CUs a late rank needed for its push (profiles/r05w_*). The ranks now see
    that they share a device and run the one-waiter form (one polling
    workgroup per rank), so the run completes on every rank."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--grid", "256",
           "--steps", "20", "--warmup", "5", "--transport", "host-peer", "--no-cpu",
           "--no-general", "--profile-steps", "0", "--force-lean",
           "--master-port", str(_port())]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = line["config"]
    assert line["n_gpus"] == 4 and line["steps"] == 20 and line["value"] > 0
    assert cfg["peer_fallback_reason"] is None, cfg["peer_fallback_reason"]
    assert cfg["transport"].startswith("peer"), cfg["transport"]
    assert cfg["peer_form"] == {"colocated": 4, "one_waiter": 1}, cfg.get("peer_form")


def test_bench_rccl_iteration_at_world_size_one():
    """--transport rccl at N = 1: the partitioned path over a one-rank RCCL
    communicator (the all-reduces run, no halo), timed as the line's value
    and reported as its rccl_iteration."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--grid", "64",
           "--steps", "20", "--warmup", "5", "--transport", "rccl", "--no-cpu", "--no-general",
           "--profile-steps", "0"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = line["config"]
    assert cfg["transport"] == "rccl"
    r = cfg["rccl_iteration"]
    assert r["iterations_per_s"] == line["iterations_per_s"] and r["ms_per_step"] > 0


def test_bench_two_ranks_auto_transport_on_one_gpu():
    """--transport auto (the driver's N > 1 default) where RCCL does not come
    up: on this one-GPU box RCCL refuses two ranks on one device, so every
    rank keeps the host transport for setup, validates the device peer
    transport against it and times the run over the peer transport."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--grid", "64",
           "--steps", "20", "--warmup", "5", "--no-cpu", "--profile-steps", "0",
           "--master-port", str(_port())]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = line["config"]
    assert cfg["rccl_note"] and "host setup transport" in cfg["rccl_note"], cfg
    assert cfg["transport_validation"]["ok"], cfg["transport_validation"]
    assert cfg["transport"] == "peer (setup: host)"
