"""bench.py driver contract on CPU: one JSON line from rank 0 with the
required keys, for 1 process and for 2 processes under torch.distributed.run
(gloo; the GPU run uses RCCL through the native engine)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _run(cmd, timeout=600, rc=0, **extra_env):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", **extra_env)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    assert (p.returncode == 0) if rc == 0 else (p.returncode == rc if rc > 0 else p.returncode != 0), \
        f"rc {p.returncode}\n" + p.stdout + p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def _check(rec, n, steps, warmup, scaling="strong", points=256 * 256):
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == n and rec["steps"] == steps and rec["warmup"] == warmup
    assert rec["value"] > 0 and rec["unit"] == "MLUPS" and rec["higher_is_better"] is True
    assert rec["dtype"] == "fp64" and rec["scaling"] == scaling
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(rec["config"])
    assert rec["config"]["global_batch"] == points


def _baseline_keys(rec, small):
    """Every BASELINE quantity is in the line, plus the correctness gate."""
    assert rec["check_max_diff"] == 0.0  # the engine is bitwise equal to the serial reference
    # the timed runs themselves, replayed through single sweeps and compared bitwise
    assert rec["timed_check_max_diff"] == 0.0 and rec["timed_check_mismatches"] == 0, rec
    assert rec[f"stencil_{small}_check_mismatches"] == 0 and "single sweeps" in rec["timed_check_path"]
    assert rec["daxpy_GBps"] > 0 and rec["daxpy_n"] > 0
    assert rec[f"stencil_{small}_MLUPS"] > 0 and "steps:" in rec[f"stencil_{small}_pass_plan"]
    assert rec["halo_exchange_us"] is not None and rec["halo_exchange_us"] > 0
    assert rec["halo_exchange_kind"]
    # BASELINE config 3: DAXPY partial sums all-reduced, checked against the closed form
    assert rec["daxpy_allsum_rel_err"] <= 1e-9
    assert rec["daxpy_allsum_exact"] == rec["n_gpus"] * (rec["daxpy_n"] + 1) / 2
    assert rec["daxpy_allreduce_us"] > 0 and rec["daxpy_partial_sum_us"] > 0
    assert rec["daxpy_allreduce_kind"]
    plan = rec["config"]["pass_plan"]
    assert plan and sum(int(a) * int(b) for a, b in (p.split("x") for p in plan.split("+"))) == rec["steps"]


def test_bench_single_process_native_engine_cpu():
    rec = _run([sys.executable, "bench.py", "--device", "cpu", "--size", "256", "--steps", "20",
                "--warmup", "5", "--daxpy-n", "20000", "--small-size", "96"])
    _check(rec, 1, 20, 5)
    assert rec["config"]["engine"] == "native"
    _baseline_keys(rec, 96)
    # N = 1: the halo latency is a labelled 1-rank periodic RCCL self-exchange
    assert "self-exchange" in rec["halo_exchange_kind"]


@pytest.mark.parametrize("transport", ["rccl", "ipc"])
def test_bench_two_ranks_torchrun_cpu(transport):
    """N = 2 under torchrun on the CPU backend; GMT_TRANSPORT=ipc runs the IPC
    transport (socket control plane + memfd emulation of the IPC kernel) that
    oversubscribed GPU ranks use."""
    port = str(free_port())
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2",
                "--device", "cpu", "--size", "256", "--steps", "3", "--warmup", "1",
                "--daxpy-n", "20000", "--ref-n-local", "32", "--ref-n-other", "300",
                "--ref-iters", "4", "--small-size", "96"], GMT_TRANSPORT=transport)
    _check(rec, 2, 3, 1)
    _baseline_keys(rec, 96)
    assert rec["config"]["engine"] == "native" and rec["config"]["transport"] == f"{transport}-host"
    assert rec["ref_halo_config"].endswith(f"{transport}-host")
    assert rec["daxpy_allreduce_kind"] == f"{transport}-host"
    assert rec["halo_exchange_us"] is not None and rec["halo_exchange_us"] > 0
    # the reference's own halo benchmark (test_deriv dim 0/1 + test_sum) on the same ranks
    assert rec["ref_halo_dim0_us"] > 0 and rec["ref_halo_dim1_us"] > 0
    assert rec["ref_halo_bytes_per_rank"] == 2 * 2 * 300 * 8 // 2  # edge ranks: one neighbour
    assert rec["ref_halo_dim0_err_norm"] < 1e-6 and rec["ref_halo_dim1_err_norm"] < 1e-6
    # every exchange's ghost rows were checked against the analytic field
    assert rec["ref_halo_dim0_bad_ghosts"] == 0 and rec["ref_halo_dim1_bad_ghosts"] == 0
    assert rec["ref_halo_dim0_rel_err"] < 1e-9 and rec["ref_halo_dim1_rel_err"] < 1e-9
    assert rec["ref_allreduce_1024_us"] > 0
    # the swapped orientation of the non-square process grid is on record too
    py, px = (int(v) for v in rec["config"]["parallelism"].split(",")[0].replace("spatial2d py", "").split(" x px"))
    assert rec["stencil_alt_dims"] == f"{px}x{py}" and rec["stencil_alt_dims_MLUPS"] > 0


def test_bench_eight_ranks_driver_shape_cpu():
    """The driver's N = 8 launch shape (one node, 8 ranks, strong scaling) on
    gloo: the 4x2 grid is timed and bitwise-gated, the swapped 2x4 grid that
    BASELINE names is timed too, and every BASELINE key is in the one line."""
    port = str(free_port())
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "8",
                "--device", "cpu", "--size", "512", "--steps", "20", "--warmup", "5",
                "--daxpy-n", "20000", "--ref-n-local", "32", "--ref-n-other", "300",
                "--ref-iters", "4", "--small-size", "128"], GMT_TRANSPORT="rccl")
    _check(rec, 8, 20, 5, points=512 * 512)
    _baseline_keys(rec, 128)
    assert rec["config"]["parallelism"].startswith("spatial2d py4 x px2")
    assert rec["stencil_alt_dims"] == "2x4" and rec["stencil_alt_dims_MLUPS"] > 0
    assert rec["ref_halo_dim0_rel_err"] < 1e-6 and rec["ref_halo_dim1_rel_err"] < 1e-6


def test_bench_two_ranks_weak_scaling_cpu():
    """--scaling weak: size x size per rank, the global domain grows with N."""
    port = str(free_port())
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2",
                "--device", "cpu", "--size", "128", "--steps", "13", "--warmup", "1",
                "--scaling", "weak", "--skip-extras"])
    _check(rec, 2, 13, 1, scaling="weak", points=2 * 128 * 128)
    assert rec["config"]["model"] == "mpi_stencil2d jacobi5 256x128 fp64"


def test_bench_overlap_autotune_keeps_the_solution():
    """--overlap auto times both modes on the real field at start-up, then
    restores the initial field: the residual after K steps is the 1-rank one."""
    common = ["--device", "cpu", "--size", "192", "--steps", "17", "--warmup", "2",
              "--daxpy-n", "2000", "--ref-n-local", "16", "--ref-n-other", "64", "--ref-iters", "2"]
    one = _run([sys.executable, "bench.py", *common])
    port = str(free_port())
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2", *common])
    tuned = two["config"]["overlap_tuning"]
    assert tuned and tuned["overlap_s"] > 0 and tuned["serial_s"] > 0
    assert abs(two["residual_l2"] - one["residual_l2"]) <= 1e-12 * max(1.0, one["residual_l2"])


def test_bench_ipc_peer_hang_fails_the_job_cpu():
    """Fault injection on the IPC transport (CPU backend): rank 1 stops at its
    3rd halo exchange; rank 0's bounded wait gives up, the engine reads the
    error word at synchronize() and aborts — the job exits non-zero with no
    JSON number (the GPU version: tests/test_multirank_gpu.py)."""
    port = str(free_port())
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               GMT_TRANSPORT="ipc", GMT_INJECT_HANG="1:2", GMT_WAIT_TIMEOUT_MS="500")
    p = subprocess.run(["timeout", "-k", "5", "120", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", port, "bench.py",
                        "--gpus", "2", "--device", "cpu", "--size", "128", "--steps", "6", "--warmup", "1",
                        "--skip-extras"], capture_output=True, text=True, timeout=150, cwd=ROOT, env=env)
    assert p.returncode != 0, p.stdout + p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")], p.stdout
    assert "GMT FAULT INJECTION: rank 1" in p.stderr, p.stderr[-4000:]
    assert "timed out waiting for the peer" in p.stdout + p.stderr, (p.stdout + p.stderr)[-4000:]


def test_bench_rccl_peer_hang_watchdog_cpu():
    """A rank that hangs inside the RCCL data plane (emulated on the CPU
    backend): rank 1 stops forever at its 3rd halo exchange, rank 0 blocks in
    the grouped send/recv.  The engine's watchdog (armed by bench.py's default
    GMT_TIMEOUT, here 4 s) ends the job with status 124 and a line naming the
    rank and its last phase, well before any launcher timeout."""
    port = str(free_port())
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               GMT_TRANSPORT="rccl", GMT_INJECT_HANG="1:2", GMT_TIMEOUT="4")
    p = subprocess.run(["timeout", "-k", "5", "150", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", port, "bench.py",
                        "--gpus", "2", "--device", "cpu", "--size", "128", "--steps", "6", "--warmup", "1",
                        "--skip-extras"], capture_output=True, text=True, timeout=180, cwd=ROOT, env=env)
    assert p.returncode != 0, p.stdout + p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")], p.stdout
    assert "GMT FAULT INJECTION: rank 1" in p.stderr, p.stderr[-4000:]
    assert "GMT WATCHDOG: rank 1" in p.stderr and "last phase" in p.stderr, p.stderr[-4000:]


def test_rccl_init_timeout_names_the_rank_cpu():
    """A communicator whose peers never join: rank 0 of 2 creates the engine's
    RCCL transport alone.  gmt_ccl_comm_init gives up after
    GMT_CCL_INIT_TIMEOUT seconds and the engine exits 124 naming the rank and
    the phase, instead of blocking the job forever."""
    code = ("import ctypes, sys; sys.path.insert(0, '.');"
            "from gpu_mpi_tests_amd import engine as e;"
            "lib = e.load('cpu'); buf = ctypes.create_string_buffer(128);"
            "assert lib.gmt_engine_unique_id(buf) == 0;"
            "lib.gmt_engine_comm_create.restype = ctypes.c_void_p;"
            "lib.gmt_engine_comm_create(0, 2, e.RCCL, buf); print('returned')")
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", GMT_CCL_INIT_TIMEOUT="2")
    env.pop("GMT_TIMEOUT", None)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=ROOT, env=env)
    assert p.returncode == 124, p.stdout + p.stderr
    assert "returned" not in p.stdout
    assert "rank 0 of 2" in p.stderr and "RCCL communicator init failed" in p.stderr, p.stderr
    assert "never" in p.stderr, p.stderr


def test_bench_transport_probe_cpu():
    """The start-up data-plane choice (bench.py --transport-probe; on the GPU
    it runs by default at one rank per GPU): an isolated child process group
    gates and times both transports (the CPU backend's RCCL socket and IPC
    memfd emulations); every candidate's exchange time is in the line and the
    job runs on the faster one."""
    port, pport = str(free_port()), str(free_port())
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2",
                "--device", "cpu", "--size", "600", "--steps", "3", "--warmup", "1", "--skip-extras",
                "--transport-probe", "on", "--probe-port", pport, "--probe-iters", "5", "--probe-passes", "2"])
    cands = rec["transport_candidates"]
    sys.path.insert(0, ROOT)
    assert set(cands) == {"rccl", "ipc", "push"}, cands
    for c in cands.values():
        assert c["gate"] == "pass" and c["pass_ms"] > 0, cands
    assert cands["rccl"]["exchange_us"] > 0 and cands["ipc"]["exchange_us"] > 0
    assert "inline halo" in cands["push"]["label"]
    chosen = {"rccl-host": "rccl", "ipc-host": "ipc", "ipc-host inline halo": "push"}[rec["config"]["transport"]]
    import bench
    assert chosen == bench.choose_plane({t: c["pass_ms"] for t, c in cands.items()})
    for c in cands.values():  # both interleaved reps on record, the better one kept
        assert len(c["pass_ms_reps"]) == 2 and c["pass_ms"] == min(c["pass_ms_reps"])
    assert rec["check_max_diff"] == 0.0 and rec["transport_probe_s"] > 0


def test_bench_transport_probe_drops_a_crashing_candidate_cpu():
    """A candidate whose probe dies (rank 1's child exits 139 at the IPC
    candidate, as a GPU memory fault would end it) is dropped: the job itself
    is untouched, runs on RCCL, and the line names the failure."""
    port, pport = str(free_port()), str(free_port())
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2",
                "--device", "cpu", "--size", "192", "--steps", "3", "--warmup", "1", "--skip-extras",
                "--transport-probe", "on", "--probe-port", pport, "--probe-iters", "5", "--probe-timeout", "20"],
               GMT_PROBE_CRASH="1:ipc")
    cands = rec["transport_candidates"]
    assert cands["rccl"]["gate"] == "pass" and cands["rccl"]["pass_ms"] > 0, cands
    assert cands["ipc"]["gate"] == "fail" and "probe exit" in cands["ipc"]["error"], cands
    assert rec["config"]["transport"] in ("rccl-host", "ipc-host inline halo") and rec["check_max_diff"] == 0.0


def test_bench_probe_drops_rccl_every_extra_on_ipc_cpu():
    """The probe's RCCL candidate dies (rank 1's child exits 139 at RCCL): the
    job, the reference halo benchmark and the DAXPY all-reduce all run on the
    surviving IPC data plane, with the extras on, and the line says why RCCL
    was dropped ("next round" item 3)."""
    port, pport = str(free_port()), str(free_port())
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2",
                "--device", "cpu", "--size", "600", "--steps", "3", "--warmup", "1",
                "--daxpy-n", "20000", "--ref-n-local", "32", "--ref-n-other", "300", "--ref-iters", "4",
                "--small-size", "96", "--transport-probe", "on", "--probe-port", pport, "--probe-iters", "5",
                "--probe-passes", "2", "--probe-timeout", "60"], GMT_PROBE_CRASH="1:rccl")
    cands = rec["transport_candidates"]
    assert cands["rccl"]["gate"] == "fail" and "probe exit 139" in cands["rccl"]["error"], cands
    assert cands["ipc"]["gate"] == "pass" and cands["push"]["gate"] == "pass", cands
    assert rec["config"]["transport"] in ("ipc-host", "ipc-host inline halo"), rec["config"]["transport"]
    assert rec["ref_halo_config"].endswith("ipc-host") and rec["daxpy_allreduce_kind"] == "ipc-host"
    assert rec["ref_halo_dim0_bad_ghosts"] == 0 and rec["daxpy_allsum_rel_err"] <= 1e-9
    assert not [k for k in rec if k.endswith("_error")], rec


def test_bench_extra_hang_keeps_the_headline_cpu():
    """An extra that hangs after the headline is measured (rank 1 stops in
    the DAXPY all-reduce, rank 0 blocks in it): the watchdog prints the line
    it was given — the headline, every extra finished before, and a
    "watchdog" field naming the stall — and every rank exits 5 (bench.py
    EXTRA_HANG_EXIT), which torchrun turns into a failed job."""
    port = str(free_port())
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2",
                "--device", "cpu", "--size", "192", "--steps", "3", "--warmup", "1",
                "--daxpy-n", "20000", "--ref-n-local", "32", "--ref-n-other", "300", "--ref-iters", "4",
                "--small-size", "0"], timeout=300, rc=-1, GMT_TRANSPORT="rccl", GMT_TIMEOUT="6",
               GMT_BENCH_HANG="1:daxpy all-reduce")
    _check(rec, 2, 3, 1, points=192 * 192)
    assert rec["check_max_diff"] == 0.0 and rec["daxpy_GBps"] > 0 and rec["ref_halo_dim0_us"] > 0
    assert "daxpy_allsum" not in rec
    assert "no progress" in rec["watchdog"] and "daxpy all-reduce" in rec["watchdog"], rec["watchdog"]


def test_bench_extra_exception_is_recorded_cpu():
    """An extra that raises is a field of the line, not an exit: a DAXPY of
    an impossible size fails alone and the job still reports."""
    rec = _run([sys.executable, "bench.py", "--device", "cpu", "--size", "128", "--steps", "4",
                "--warmup", "1", "--daxpy-n", "-5", "--small-size", "0"])
    _check(rec, 1, 4, 1, points=128 * 128)
    assert "daxpy_error" in rec and "daxpy_all-reduce_error" in rec, sorted(rec)
    assert rec["halo_exchange_us"] > 0


def test_bench_extra_hang_exit_status_single_process_cpu():
    """N = 1 (no launcher in between): a hung extra exits with bench.py's
    EXTRA_HANG_EXIT (5) after printing the headline line."""
    rec = _run([sys.executable, "bench.py", "--device", "cpu", "--size", "128", "--steps", "4", "--warmup", "1",
                "--daxpy-n", "20000", "--small-size", "0"], timeout=120, rc=5, GMT_TIMEOUT="4",
               GMT_BENCH_HANG="0:daxpy all-reduce")
    assert rec["timed_check_mismatches"] == 0 and "daxpy all-reduce" in rec["watchdog"]


@pytest.mark.parametrize("ranks", [1, 2, 4])
def test_bench_timed_check_catches_a_corrupt_face_cpu(ranks):
    """The check of the timed run: rank R
    overwrites one ghost cell of its input at the 2nd fused pass of the timed
    run — at N > 1 a cell the inline halo (push) stored from the neighbour —
    and the single-sweep replay differs, so the job exits non-zero with the
    mismatch in the line (no small-domain gate: --skip-check; table-planned
    fused passes: --no-calibrate)."""
    args = ["bench.py", "--gpus", str(ranks), "--device", "cpu", "--size", "600", "--steps", "20",
            "--warmup", "5", "--skip-check", "--no-calibrate", "--skip-extras"]
    if ranks > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), *args, "--transport", "push"]
    else:
        cmd = [sys.executable, *args]
    clean = _run(cmd, timeout=300)
    assert clean["timed_check_mismatches"] == 0 and clean["timed_check_max_diff"] == 0.0
    if ranks > 1:
        assert clean["config"]["transport"] == "ipc-host inline halo", clean["config"]
    bad = _run(cmd, timeout=300, rc=6 if ranks == 1 else -1, GMT_CORRUPT_PASS=f"{ranks - 1}:2")
    assert bad["timed_check_mismatches"] > 0 and bad["timed_check_max_diff"] > 0, bad
    assert bad["timed_check_failed"] == ["timed_check"]


def test_probe_order_and_margin():
    """candidates are timed interleaved (A B C C B
    A), and a more involved data plane must beat the simpler one it replaces
    by more than 3% (rccl < ipc < push); a tie keeps the simpler plane."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench.probe_order(["rccl", "ipc", "push"]) == [("rccl", 0), ("ipc", 0), ("push", 0),
                                                          ("push", 1), ("ipc", 1), ("rccl", 1)]
    pick = bench.choose_plane
    assert pick({"rccl": 1.00, "ipc": 0.98, "push": 0.975}) == "rccl"   # all within 3%: simplest
    assert pick({"rccl": 1.00, "ipc": 0.96, "push": 0.95}) == "ipc"     # push within 3% of ipc
    assert pick({"rccl": 1.00, "ipc": 0.96, "push": 0.92}) == "push"
    assert pick({"rccl": 1.00, "ipc": 1.20, "push": 0.96}) == "push"
    assert pick({"ipc": 1.00, "push": 0.98}) == "ipc"                   # ranks sharing a GPU: no rccl
    assert pick({"ipc": 1.00, "push": 0.96}) == "push"
    assert pick({"push": 1.0}) == "push" and pick({}) == "auto"


def test_bench_push_stalled_neighbour_stops_the_passes_cpu():
    """an inline-halo hand-over that times out stops
    every later pass at once (gmt_push_sync sets the stop word the passes
    check at entry; later hand-overs neither signal nor wait) and the job
    aborts at the next synchronisation.  Rank 1 stalls at its 11th exchange (a hand-over)
    (GMT_INJECT_HANG); rank 0's wait gives up after 2 s.  Without the stop
    every one of the ~40 passes left would wait its own 2 s."""
    import time
    port = str(free_port())
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               GMT_INJECT_HANG="1:10", GMT_WAIT_TIMEOUT_MS="2000")
    t0 = time.time()
    p = subprocess.run(["timeout", "-k", "5", "200", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", port, "bench.py",
                        "--gpus", "2", "--device", "cpu", "--size", "600", "--steps", "800", "--warmup", "1",
                        "--skip-extras", "--skip-check", "--no-calibrate", "--transport", "push"],
                       capture_output=True, text=True, timeout=230, cwd=ROOT, env=env)
    dt = time.time() - t0
    out = p.stdout + p.stderr
    assert p.returncode != 0, out[-3000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")], p.stdout
    assert "GMT FAULT INJECTION: rank 1" in p.stderr, out[-3000:]
    assert "inline-halo hand-over timed out" in out, out[-3000:]
    assert dt < 60, dt  # one expired wait, not one per remaining pass
