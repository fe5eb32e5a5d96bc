#!/usr/bin/env python3
"""Flagship benchmark: distributed 2-D 5-point Jacobi (fp64) on MI355X.

Metric (BASELINE.json): "DAXPY GB/s + 2D stencil MLUPS at 1/2/4/8 MI355X;
halo-exchange latency".  The headline ``value`` is the whole-job stencil rate
in MLUPS (million lattice-point updates per second, summed over all GPUs) on
the BASELINE multi-GPU config "mpi_stencil2d 32768² ... (2×4 decomp), halo
exchange/interior overlap".  The global domain is FIXED at 32768² for every N
(strong scaling: N = 8 is exactly the named config).  The same JSON line
carries every other BASELINE quantity:

* ``stencil_8192_MLUPS``: the same engine on the 8192² domain (BASELINE
  "mpi_stencil2d 8192² fp64 single GPU" at N = 1);
* ``daxpy_GBps``: DAXPY N = 2^28 fp64 per GPU (BASELINE "daxpy N=2^28");
* ``halo_exchange_us``: one blocking K-wide halo exchange of the 32768² field
  (N > 1: the job's own exchange over RCCL/xGMI; N = 1: a 1-rank periodic
  RCCL self-exchange of the same faces, labelled in ``halo_exchange_kind``);
* N > 1: the reference's own halo benchmark (``ref_halo_*``, test_deriv /
  test_sum of mpi_stencil2d_gt) over RCCL.

One step = one full Jacobi sweep of the global domain (every point updated
once).  The native engine (C++, ``csrc/engine/jacobi.cpp``) runs the steps in
fused passes of up to ``--tsteps`` sweeps (temporal blocking with
``csrc/kernels/jacobi5tb.hip``): one K-wide halo exchange (RCCL over xGMI on a
high-priority stream, overlapped with the core of the pass) and one pass that
reads u(t) once and writes u(t+K) once — bitwise the same result as K single
sweeps.  ``JacobiSolver::plan_passes`` splits the timed steps into the
cheapest sequence of passes; the JSON reports that plan (``pass_plan``), and
every pass type of it is launched once before the warm-up
(``NativeJacobi.prepare``), so no first launch lands in the timed region.
Nothing is skipped inside the timed region: K steps are K sweeps of every
lattice point.

Before timing, every run checks its decomposition: the engine with the same
process grid and K runs a small domain and is compared with the serial NumPy
reference (``check_max_diff``, must be 0 — the engine is bitwise); a
mismatch exits non-zero.

Launch (driver contract):
    python bench.py --gpus 1 --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DEFAULT_TSTEPS = 20  # max fused sweeps per memory pass / halo exchange; the engine plans the mix (profiles/r02_tb.md)

from gpu_mpi_tests_amd import ops  # noqa: E402
from gpu_mpi_tests_amd.engine import MAX_TSTEPS, watchdog_epitaph, watchdog_timeout  # noqa: E402
from gpu_mpi_tests_amd.parallel import dist as gdist  # noqa: E402
from gpu_mpi_tests_amd.parallel.decomp import choose_dims  # noqa: E402


def mark(env, phase):
    """Progress mark for the engine's hang watchdog (armed by the first engine
    call; GMT_TIMEOUT seconds without a mark end the job with status 124 and a
    line naming the rank and this phase)."""
    from gpu_mpi_tests_amd.engine import watchdog_kick

    watchdog_kick(f"bench.py: {phase}", "cuda" if env.is_gpu else "cpu")


def _sync(env):
    if env.is_gpu:
        torch.cuda.synchronize(env.device)


def _timed(env, fn_run, fn_sync, steps, warmup, on_start=None):
    fn_run(warmup)
    fn_sync()
    gdist.barrier(env)
    _sync(env)
    if on_start is not None:
        on_start()  # stream ordered (the engine's clock record reset): after the warm-up
    t0 = time.perf_counter()
    fn_run(steps)
    fn_sync()
    _sync(env)
    # this rank's finish, read before the closing barrier (whose own cost is
    # not part of the K steps); the job's time is the max over ranks
    dt = time.perf_counter() - t0
    gdist.barrier(env)
    return gdist.allreduce_max(dt, env)


def plan_str(plan):
    """[14, 14, 12] -> '2x14+1x12' (sweeps per fused pass, launch order grouped)."""
    out, i = [], 0
    while i < len(plan):
        j = i
        while j < len(plan) and plan[j] == plan[i]:
            j += 1
        out.append(f"{j - i}x{plan[i]}")
        i = j
    return "+".join(out)


def _plane(plane):
    """A data plane of the probe / --transport -> (engine transport, push):
    "push" is the IPC transport with the inline halo exchange (each fused
    pass stores its faces straight into the neighbours' ghost cells,
    gmt/jacobi.hpp JacobiConfig::push)."""
    return ("ipc", True) if plane == "push" else (plane, False)


def bench_native(env, shape, steps, warmup, overlap, dims, graph, tblock, wg_waves, seg_rows, init="random",
                 seed=0, calibrate=True, transport="auto"):
    from gpu_mpi_tests_amd.engine import NativeJacobi

    t, push = _plane(transport)
    eng = NativeJacobi(shape[0], shape[1], env, dims=dims, overlap=overlap, graph=graph, tblock=tblock,
                       wg_waves=wg_waves, seg_rows=seg_rows, init=init, seed=seed, calibrate=calibrate,
                       transport=t, push=push and env.world_size > 1)
    # calibration (one timed pass of every pass size on this share, max over
    # ranks) -> the plan; then one launch of every pass type of the timed
    # plan; the initial field is restored
    eng.prepare(steps)
    dt = _timed(env, eng.run, eng.synchronize, steps, warmup, on_start=eng.clock_reset)
    clk = eng.clock()
    # min over ranks: the slowest clock of the job
    info = {"clock": {"sclk_mhz": -gdist.allreduce_max(-clk["sclk_mhz"], env), "samples": clk["samples"]},
            "engine": "native", "graph": eng.graph, "overlap": eng.overlap, "tblock": eng.tblock,
            "overlap_tuning": eng.tuned, "tsteps": eng.tsteps, "pass_plan": plan_str(eng.plan(steps)),
            "exact": eng.exact, "max_abs_u0": eng.max_abs_u0, "pass_cost_ms": eng.pass_cost_ms(),
            "transport": (eng.transport + (" inline halo" if eng.push_active else "")
                          if env.world_size > 1 else "none"),
            "halo_bytes_per_rank": eng.halo_bytes, "dims": (eng.py, eng.px),
            "tb_launch": eng.tb_launch(eng.tsteps) if eng.tblock and eng.tsteps > 1 else None}
    return eng, dt, info


def timed_check(env, eng, sweeps, init, seed, prefix="timed_check"):
    """The check of the timed run itself, on the timed domain (reference: the
    timed field's err_norm, mpi_stencil2d_gt.cc:541-570).  The same initial
    field is advanced by the same sweeps (warm-up + timed) through an
    independent path — single sweeps (csrc/kernels/jacobi5.hip) with one plain
    blocking 1-wide halo exchange per sweep over RCCL (IPC when ranks share a
    GPU, none at N = 1): no fused passes, no segment plan, no inline halo, no
    overlap — and the two final interiors are compared bitwise on the device
    (gmt_diff_bits; max |diff| and differing elements over ranks).  Must be
    0 / 0: the fused passes are bitwise equal to single sweeps."""
    from gpu_mpi_tests_amd.engine import NativeJacobi

    t0 = time.perf_counter()
    if env.world_size == 1:
        t = "auto"
    else:
        t = "ipc" if env.is_gpu and env.ranks_per_device > 1 else "rccl"
    ref = NativeJacobi(eng.ny_g, eng.nx_g, env, dims=(eng.py, eng.px), overlap=False, graph=False, tblock=False,
                       init=init, seed=seed, transport=t)
    try:
        ref.run(sweeps)
        ref.synchronize()
        eng.synchronize()
        mx, bad = eng.compare(ref)
        kind = ref.transport
    finally:
        ref.close()
    if env.is_gpu:
        torch.cuda.empty_cache()
    return {f"{prefix}_max_diff": mx, f"{prefix}_mismatches": bad,
            f"{prefix}_path": f"{sweeps} single sweeps + blocking 1-wide exchange ({kind}), bitwise on the device",
            f"{prefix}_s": round(time.perf_counter() - t0, 3)}


def check_engine(env, dims, tsteps, graph, init="analytic", seed=0, transport="auto"):
    """Distributed-correctness gate (reference: mpi_stencil2d_gt.cc:555-570
    err_norm): the engine with this job's process grid and sweeps per pass on
    a small Dirichlet domain, overlap on and off, vs the serial NumPy
    reference.  Returns the max |difference| over both runs (0 = bitwise)."""
    from gpu_mpi_tests_amd.engine import NativeJacobi, serial_jacobi

    from gpu_mpi_tests_amd.engine import group_cols

    py, px = dims
    k = max(1, tsteps)
    t, push = _plane(transport)
    # every rank big enough for the overlapped (band-first) pass: K-deep
    # bands plus an interior in y, three workgroup-wide strips in x
    wb = group_cols(k, 0, "cuda" if env.is_gpu else "cpu") if k > 1 else 0
    ny, nx = py * (4 * k + 75) + 3, px * (3 * wb + 8 * k + 37) + 5
    steps = 2 * k + 3  # full passes, a remainder pass and (odd) single sweeps
    ref = serial_jacobi(ny, nx, steps, init=init, seed=seed) if env.rank == 0 else None
    worst = 0.0
    for ov in ((True,) if push else (True, False)):
        e = NativeJacobi(ny, nx, env, dims=dims, overlap=ov, graph=graph, tblock=k if k > 1 else False,
                         init=init, seed=seed, transport=t, push=push)
        if push and not e.push_active:
            # the gate must check the plane the job will run, not the
            # transport's exchange it would fall back to
            e.close()
            raise RuntimeError(f"the inline halo exchange does not apply to the gate's {ny}x{nx} shares")
        e.run(steps)
        e.synchronize()
        part = (e.off_y, e.off_x, e.interior())
        e.close()
        if env.world_size > 1:
            parts = [None] * env.world_size
            torch.distributed.all_gather_object(parts, part, group=env.host_group)
        else:
            parts = [part]
        if env.rank == 0:
            full = np.full((ny, nx), np.nan)
            for oy, ox, a in parts:
                full[oy:oy + a.shape[0], ox:ox + a.shape[1]] = a
            worst = max(worst, float(np.nanmax(np.abs(full - ref))) if not np.isnan(full).any() else float("inf"))
    return gdist.allreduce_max(worst, env)


def peer_status(env, dims):
    """Which process-grid neighbours' GPUs this rank's GPU can reach directly
    (xGMI peer access), gathered on rank 0: {"peer_access": bool, "rccl": version,
    "ranks_per_gpu": n}.  Neighbours on the same GPU (oversubscription) need none."""
    if not env.is_gpu or env.world_size == 1:
        return {}
    py, px = dims
    cy, cx = divmod(env.rank, px)
    nbrs = [(cy + dy) * px + (cx + dx) for dy, dx in ((-1, 0), (1, 0), (0, -1), (0, 1))
            if 0 <= cy + dy < py and 0 <= cx + dx < px]
    ok = True
    for r in nbrs:
        # single node, block mapping (parallel/dist.py select_device): rank r on r // ranks_per_device
        dev = (r // max(1, env.ranks_per_device)) % max(1, env.n_devices)
        if dev != env.device.index:
            ok = ok and bool(torch.cuda.can_device_access_peer(env.device.index, dev))
    flags = [None] * env.world_size
    torch.distributed.all_gather_object(flags, ok, group=env.host_group)
    ver = torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else None
    return {"peer_access": all(flags), "rccl_version": ".".join(map(str, ver)) if isinstance(ver, tuple) else ver,
            "ranks_per_gpu": env.ranks_per_device}


def halo_latency(env, eng, iters):
    """Blocking halo exchange of the engine's current field: mean seconds (max over ranks)."""
    for _ in range(5):
        eng.exchange()
    _sync(env)
    gdist.barrier(env)
    t0 = time.perf_counter()
    for _ in range(iters):
        eng.exchange()
    _sync(env)
    dt = (time.perf_counter() - t0) / iters
    return gdist.allreduce_max(dt, env)


def self_halo_latency(env, shape, tsteps, iters):
    """N = 1: the same K-wide faces of the same field exchanged by a 1-rank
    periodic engine with itself over RCCL (send/recv to self)."""
    from gpu_mpi_tests_amd.engine import NativeJacobi

    eng = NativeJacobi(shape[0], shape[1], env, periodic=True, overlap=False, graph=False,
                       tblock=tsteps if tsteps > 1 else False, transport="rccl")
    try:
        return halo_latency(env, eng, iters), eng.halo_bytes, eng.transport
    finally:
        eng.close()


def ref_halo(env, n_local, n_other, iters, transport="auto", check_iters=20):
    """The reference's own headline measurement (mpi_stencil2d_gt test_deriv /
    test_sum: 2-deep ghost faces of n_other doubles — 8 MiB at the defaults —
    exchanged between 1-D slab neighbours, dim 0 packed, dim 1 in place, the
    derivative kernel after each exchange; then the 1024-double all-reduce),
    over this job's transport (RCCL; IPC when ranks share a GPU).  Per-exchange
    median, max over ranks.  The timed run is the reference's loop as is; a
    separate untimed run of ``check_iters`` exchanges raises the field before
    every exchange and checks every ghost cell after it (gmt/deriv.hpp)."""
    from gpu_mpi_tests_amd.engine import deriv_bench

    r = deriv_bench(n_local, n_other, n_iter=iters, n_warmup=5, env=env, check=False, transport=transport)
    rc = deriv_bench(n_local, n_other, n_iter=check_iters, n_warmup=1, env=env, check=True, transport=transport)
    out = {"ref_halo_config": f"mpi_stencil2d_gt {n_local}x{n_other} per rank, 1-D slabs, "
                              f"{iters} timed exchanges + {check_iters} checked untimed, {r['transport']}"}
    for d in (0, 1):
        out[f"ref_halo_dim{d}_us"] = round(gdist.allreduce_max(r[f"dim{d}"]["median_s"], env) * 1e6, 2)
        out[f"ref_halo_dim{d}_err_norm"] = gdist.allreduce_max(r[f"dim{d}"]["err_norm"], env)
        # every checked exchange's ghost rows vs the analytic field
        out[f"ref_halo_dim{d}_bad_ghosts"] = int(gdist.allreduce_max(float(rc[f"dim{d}"]["bad_ghosts"]), env))
        # scale-free: round-off of x^3 + y^2 at the reference's spacing grows
        # with the extent; a missing or wrong ghost cell gives O(1) and more
        out[f"ref_halo_dim{d}_rel_err"] = gdist.allreduce_max(
            r[f"dim{d}"]["err_norm"] / max(r[f"dim{d}"]["exact_norm"], 1e-300), env)
    out["ref_halo_bytes_per_rank"] = int(gdist.allreduce_max(float(r["dim0"]["bytes"]), env))
    out["ref_allreduce_1024_us"] = round(gdist.allreduce_max(r["allreduce_median_s"], env) * 1e6, 2)
    return out


def bench_daxpy(env, n, iters):
    """Per-GPU DAXPY rate (each rank on its own GPU, random-init x and y),
    reported as whole-job GB/s."""
    dev = env.device
    x = torch.rand(n, dtype=torch.float64, device=dev)
    y = torch.rand(n, dtype=torch.float64, device=dev)
    for _ in range(3):
        ops.daxpy(2.0, x, y)
    _sync(env)
    gdist.barrier(env)
    if env.is_gpu:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            ops.daxpy(2.0, x, y)
        e1.record()
        e1.synchronize()
        dt = e0.elapsed_time(e1) / 1e3 / iters
    else:
        t0 = time.perf_counter()
        for _ in range(iters):
            ops.daxpy(2.0, x, y)
        dt = (time.perf_counter() - t0) / iters
    dt = gdist.allreduce_max(dt, env)
    del x, y
    return 24.0 * n / dt / 1e9 * env.world_size, dt


def daxpy_allreduce(env, n, iters, transport="auto"):
    """BASELINE config "mpi_daxpy N ranks x 1 GPU, RCCL allreduce of partial
    sums": the reference's distributed DAXPY check (mpi_daxpy_nvtx.cc:207-310)
    with its closed form — x = (i+1)/n, y = -x, y <- 2x + y = x, so each rank's
    SUM = (n+1)/2 and ALLSUM = world*(n+1)/2 — where the reference's host
    sums and Allgather become a device partial sum (gfx950 reduce kernel) and
    an in-place all-reduce of it over the native transport (RCCL over xGMI;
    IPC when ranks share a GPU; a labelled 1-rank self all-reduce at N = 1).
    Returns the keys for the JSON line; rel_err > 1e-9 fails the run."""
    from gpu_mpi_tests_amd.engine import Comm

    dev = env.device
    x = torch.empty(n, dtype=torch.float64, device=dev)
    ops.fill_poly(x, 3, 1.0 / n, 1.0 / n, 0.0, 0.0)  # x[i] = (i+1)/n
    y = -x
    ops.daxpy(2.0, x, y)
    comm = Comm(env, transport)
    part = torch.empty(1, dtype=torch.float64, device=dev)
    t_sum, t_red = [], []
    try:
        for i in range(iters + 3):
            _sync(env)
            t0 = time.perf_counter()
            ops.vsum(y, out=part)  # this rank's SUM, on the device (one HBM pass)
            _sync(env)
            t1 = time.perf_counter()
            allsum = part.clone()
            _sync(env)
            t2 = time.perf_counter()
            comm.allreduce_sum_(allsum)
            t3 = time.perf_counter()
            if i >= 3:
                t_sum.append(t1 - t0)
                t_red.append(t3 - t2)
        local, total = float(part.item()), float(allsum.item())
    finally:
        comm.close()
    exact_local = (n + 1) / 2.0
    exact = env.world_size * exact_local
    rel = max(abs(total - exact) / exact, gdist.allreduce_max(abs(local - exact_local) / exact_local, env))
    kind = comm.name if env.world_size > 1 else f"1-rank self all-reduce ({comm.name})"
    del x, y
    return {"daxpy_allsum": total, "daxpy_allsum_exact": exact, "daxpy_allsum_rel_err": rel,
            "daxpy_partial_sum_us": round(gdist.allreduce_max(float(np.median(t_sum)), env) * 1e6, 2),
            "daxpy_allreduce_us": round(gdist.allreduce_max(float(np.median(t_red)), env) * 1e6, 2),
            "daxpy_allreduce_kind": kind}


PROBE_KINDS = ("rccl", "ipc", "push")


def _env_transport():
    """The engine transport an environment variable forces, or ''."""
    eng = os.environ.get("GMT_ENGINE_TRANSPORT", "").strip().lower()
    app = os.environ.get("GMT_TRANSPORT", "").strip().lower()
    return eng if eng not in ("", "auto") else (app if app in PROBE_KINDS else "")


def probe_kinds(args):
    """Data planes to time at start-up (before this process touches the GPU).
    auto: N > 1 with every rank on its own GPU, where both RCCL and IPC (peer
    mappings over xGMI) can carry the halo; on: also on the CPU backend (its
    socket / memfd emulations) or with ranks sharing a GPU (IPC only)."""
    world = int(os.environ.get("WORLD_SIZE", "1") or 1)
    if world < 2 or args.transport != "auto" or args.transport_probe == "off" or _env_transport():
        return []
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)) or world)
    ndev = 0 if args.device == "cpu" else torch.cuda.device_count()  # counting does not initialise the GPU
    if args.transport_probe == "on":
        return list(PROBE_KINDS) if ndev == 0 or lw <= ndev else ["ipc", "push"]
    return list(PROBE_KINDS) if 0 < ndev and lw <= ndev else []


def probe_order(kinds):
    """Interleaved rep order of the probe's candidates: A B C C B A.  The
    clock drifts over a sustained run (the first of a pair reads high,
    profiles/r05_overlap/README.md), so every candidate is timed once early
    and once late, and keeps its better rep."""
    return [(k, 0) for k in kinds] + [(k, 1) for k in reversed(kinds)]


def run_probe(args, argv, kinds):
    """Time every candidate data plane in a CHILD process group of its own
    (this process has not initialised the GPU yet): a candidate that faults,
    hangs or fails the bitwise gate takes only its child down and is
    dropped, never the job nor the other candidates.  Each candidate runs
    twice, in the interleaved order of probe_order; each child rendezvouses
    on its own port and is killed as a process group at --probe-timeout.
    Returns this rank's candidates ({kind: {"reps": [rec, rec]}}, each rec
    with its child's exit status) and the probe's wall time."""
    import signal
    import subprocess
    import tempfile

    rank = int(os.environ.get("RANK", "0") or 0)
    port = int(os.environ.get("MASTER_PORT", "29500") or 29500)
    order = probe_order(kinds)
    base = args.probe_port or (port + 101 if port + 101 + len(order) < 65536 else port - 101 - len(order))
    res = {k: {"reps": [None, None]} for k in kinds}
    t0 = time.perf_counter()
    for i, (kind, rep) in enumerate(order):
        cenv = dict(os.environ, MASTER_PORT=str(base + i), GMT_TIMEOUT=str(min(60.0, args.probe_timeout)))
        # torchrun's agent hosts the store on MASTER_PORT only: the children host their own
        cenv.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        fd, path = tempfile.mkstemp(prefix=f"gmt_probe_r{rank}_{kind}{rep}_", suffix=".json")
        os.close(fd)
        cmd = [sys.executable, os.path.abspath(__file__), *argv, "--probe-child", path, "--probe-kinds", kind]
        t1 = time.perf_counter()
        p = subprocess.Popen(cmd, stdout=sys.stderr, start_new_session=True, env=cenv)
        try:
            rc = p.wait(timeout=args.probe_timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)  # the child's own session: exactly the process group started here
            p.wait()
            rc = "timeout"
        rec = {}
        try:
            with open(path) as f:
                txt = f.read()
            rec = (json.loads(txt) if txt else {}).get(kind, {})
        except (OSError, ValueError) as ex:
            rc = f"{rc}, unreadable result: {ex}"
        finally:
            os.unlink(path)
        rec["_rc"] = rc
        rec["_s"] = round(time.perf_counter() - t1, 2)
        res[kind]["reps"][rep] = rec
    res["_s"] = round(time.perf_counter() - t0, 2)
    return res


def probe_pass_ms(env, eng, tsteps, passes):
    """ms per fused pass of the engine as built (exchange or inline halo, and
    overlap, included), max over ranks: what the candidate costs the run."""
    eng.run(tsteps)
    eng.synchronize()
    gdist.barrier(env)
    t0 = time.perf_counter()
    eng.run(passes * tsteps)
    eng.synchronize()
    dt = (time.perf_counter() - t0) / passes
    return gdist.allreduce_max(dt, env) * 1e3


def probe_child(args, dims, shape, tsteps, graph):
    """--probe-child: the candidate's bitwise gate on this process grid, then
    the cost of its fused passes on the headline field (``pass_ms``: the
    passes as the job would run them, exchange or inline halo included, mean
    over --probe-passes, max over ranks) and, for the exchange transports,
    the blocking K-wide exchange (mean over --probe-iters), written as JSON
    to the given path.  Fault injection: GMT_PROBE_CRASH=R:KIND makes rank R's
    child die (status 139, as on a GPU memory fault) when it reaches KIND."""
    from gpu_mpi_tests_amd.engine import NativeJacobi

    env = gdist.init(device=args.device)
    crash = os.environ.get("GMT_PROBE_CRASH", "").split(":")
    out = {}
    for plane in args.probe_kinds.split(","):
        mark(env, f"transport probe: {plane}")
        if len(crash) == 2 and crash[0] == str(env.rank) and crash[1] == plane:
            print(f"GMT FAULT INJECTION: rank {env.rank} transport probe child dies at {plane}", file=sys.stderr,
                  flush=True)
            os._exit(139)
        t, push = _plane(plane)
        rec = {}
        try:
            rec["gate_max_diff"] = check_engine(env, dims, tsteps, graph, "analytic", 0, transport=plane)
            if rec["gate_max_diff"] == 0.0:
                eng = NativeJacobi(shape[0], shape[1], env, dims=dims, overlap=False if push else "auto",
                                   graph=False, tblock=tsteps if tsteps > 1 else False, transport=t, push=push,
                                   calibrate=False)
                try:
                    if push and not eng.push_active:
                        raise RuntimeError("the inline halo exchange does not apply to this share")
                    rec["pass_ms"] = round(probe_pass_ms(env, eng, max(tsteps, 1), args.probe_passes), 4)
                    if not push:
                        rec["exchange_us"] = round(halo_latency(env, eng, args.probe_iters) * 1e6, 2)
                    rec["label"] = eng.transport + (" inline halo" if push else "")
                    rec["overlap"] = eng.overlap
                finally:
                    eng.close()
        except Exception as ex:  # a failing candidate is data, not a crash
            rec["error"] = f"{type(ex).__name__}: {ex}"[:300]
        out[plane] = rec
        with open(args.probe_child, "w") as f:
            json.dump(out, f)
    gdist.shutdown()


SIMPLICITY = ("rccl", "ipc", "push")  # a tie keeps the earlier (simpler) data plane


def choose_plane(pass_ms, margin=0.97):
    """{kind: pass ms} of the candidates that passed -> the job's plane.
    Candidates are visited from the simplest (RCCL: the library's own
    collectives, no mappings) to the most involved (push: the pass stores
    into peer memory); a more involved one replaces the current choice only
    when its passes are faster by more than 1 - margin (3%) — the run-to-run
    spread of a probe rep — so a tie keeps the simpler plane."""
    choice = None
    for t in sorted(pass_ms, key=lambda k: SIMPLICITY.index(k) if k in SIMPLICITY else len(SIMPLICITY)):
        if choice is None or pass_ms[t] < margin * pass_ms[choice]:
            choice = t
    return choice or "auto"


def agree_transport(env, probe, kinds, margin=0.97):
    """Every rank's probe -> one choice for all: a candidate counts if it
    passed the gate and timed on EVERY rank in BOTH of its reps; a rep's pass
    time is the max over ranks, the candidate's the better of its two reps
    (``pass_ms_reps`` records both); the plane is then choose_plane's.
    Every rank calls this (world > 1), probed or not, so ranks whose
    environments disagree on probing (device counts, LOCAL_WORLD_SIZE)
    cannot leave one side waiting in the collective: only kinds that every
    rank probed count.  Returns (transport, {kind: record} or None, probe
    wall seconds)."""
    allp = [None] * env.world_size
    torch.distributed.all_gather_object(allp, {"kinds": list(kinds), "probe": probe or {}}, group=env.host_group)
    common = [t for t in kinds if all(t in (p["kinds"] or []) for p in allp)]
    if not any(p["kinds"] for p in allp):
        return "auto", None, 0.0
    allp_kinds = {tuple(p["kinds"]) for p in allp}
    allp = [p["probe"] for p in allp]
    cands = {}
    if len(allp_kinds) > 1:
        cands["_mismatch"] = {"gate": "fail", "error": f"ranks probed different kinds: {sorted(allp_kinds)}"}
    for t in common:
        # per rank, per rep
        reps = [[r or {} for r in ((p.get(t) or {}).get("reps") or [None, None])] for p in allp]
        ok = all(r.get("gate_max_diff") == 0.0 and r.get("pass_ms") for rr in reps for r in rr)
        c = {"gate": "pass" if ok else "fail"}
        if ok:
            c["pass_ms_reps"] = [max(rr[i]["pass_ms"] for rr in reps) for i in range(2)]
            c["pass_ms"] = min(c["pass_ms_reps"])
            if all(r.get("exchange_us") for rr in reps for r in rr):
                c["exchange_us"] = min(max(rr[i]["exchange_us"] for rr in reps) for i in range(2))
            c["label"] = reps[0][0].get("label", t)
        else:
            whys = []
            for i, rr in enumerate(reps):
                why = []
                for j, r in enumerate(rr):
                    if r.get("_rc", 0) != 0:
                        why.append(f"rep {j + 1} probe exit {r.get('_rc')}")
                    if r.get("error"):
                        why.append(r["error"])
                    elif r.get("gate_max_diff"):
                        why.append(f"gate max diff {r['gate_max_diff']}")
                if why:
                    whys.append(f"rank {i}: {', '.join(why)}")
            c["error"] = "; ".join(whys[:4])[:600]
        cands[t] = c
    passing = {t: c["pass_ms"] for t, c in cands.items() if c["gate"] == "pass" and not t.startswith("_")}
    choice = choose_plane(passing, margin) if passing else "auto"
    return choice, cands, max(float(p.get("_s", 0.0)) for p in allp)


def result_record(args, env, shape, mlups, ms_per_step, info, dims):
    """The driver's JSON line without its extras (``line()`` merges them)."""
    py, px = dims
    points = shape[0] * shape[1]
    rec = {
        "metric": "2D 5-pt Jacobi stencil MLUPS (fp64)",
        "value": round(mlups, 1),
        "unit": "MLUPS",
        "n_gpus": env.world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "fp64",
        "data": (f"synthetic: random-init field, uniform [0,1) hashed from the global lattice point "
                 f"(seed {args.seed}), Dirichlet boundary" if args.init == "random" else
                 "synthetic: analytic x^3+y^2 initial field, Dirichlet boundary"),
        "config": {
            "model": f"mpi_stencil2d jacobi5 {shape[0]}x{shape[1]} fp64",
            "global_batch": points,
            "seq_len": None,
            "parallelism": f"spatial2d py{py} x px{px}, "
                           f"{'overlap' if info['overlap'] else 'serial'}",
            "engine": info["engine"],
            "hipgraph": info["graph"],
            "overlap_tuning": info.get("overlap_tuning"),
            "temporal_blocking": info["tblock"],
            "sweeps_per_pass": info.get("tsteps", 1),
            "pass_plan": info.get("pass_plan"),
            "exact_levels": info.get("exact"),
            "init": args.init,
            "max_abs_u0": info.get("max_abs_u0"),
            "pass_cost_ms": info.get("pass_cost_ms"),
            "tb_launch": info.get("tb_launch"),
            "transport": info["transport"],
            "halo_bytes_per_rank": info["halo_bytes_per_rank"],
            "device": str(env.device),
        },
    }

    return rec


def _epitaph(env, rec):
    """Returns a function that (re)registers the current result line (``rec()``)
    as the watchdog's last words (rank 0; the other ranks exit 0 silently)."""
    dev = "cuda" if env.is_gpu else "cpu"

    def update():
        watchdog_epitaph(json.dumps(rec()) if env.rank == 0 else "", EXTRA_HANG_EXIT, dev)

    return update


def _maybe_hang(env, phase):
    """Fault injection for the extras' isolation test: GMT_BENCH_HANG=R:PHASE
    makes rank R stop forever when it reaches PHASE (a substring of the phase
    name); the other ranks block in that phase's collective."""
    spec = os.environ.get("GMT_BENCH_HANG", "")
    r, _, ph = spec.partition(":")
    if spec and r == str(env.rank) and ph and ph in phase:
        print(f"GMT FAULT INJECTION: rank {env.rank} hangs in bench phase '{phase}'", file=sys.stderr, flush=True)
        while True:
            time.sleep(3600)


class TimedCheckFailed(RuntimeError):
    pass


def checked(extras, rec):
    """Merges a timed_check record; a mismatch fails the job (after the line
    is printed, bench.py exits TIMED_CHECK_EXIT)."""
    extras.update(rec)
    prefix = next(k for k in rec if k.endswith("_mismatches"))[:-len("_mismatches")]
    if rec[f"{prefix}_mismatches"] != 0 or rec[f"{prefix}_max_diff"] != 0.0:
        extras["timed_check_failed"] = sorted(set(extras.get("timed_check_failed", [])) | {prefix})
        raise TimedCheckFailed(f"{prefix}: {rec[f'{prefix}_mismatches']} lattice points differ from the "
                               f"single-sweep replay (max |diff| {rec[f'{prefix}_max_diff']})")


TIMED_CHECK_EXIT = 6  # a timed field differs from its single-sweep replay
EXTRA_HANG_EXIT = 5   # the headline stands, an extra hung (the watchdog printed the line)


def run_extras(args, env, solver, info, shape, points, tsteps, overlap, dims, graph, transport, extras, epitaph):
    """Every BASELINE quantity besides the headline, each failure-isolated:
    an exception is recorded as "<name>_error" and the next extra runs (a
    hang is the watchdog's, see main).  The data-plane extras run on the
    transport the job runs on (the probe's choice when it dropped one)."""
    iters = max(20, min(args.steps, 200))

    def extra(name, fn):
        mark(env, name)
        _maybe_hang(env, name)
        try:
            fn()
        except Exception as ex:  # isolated: the line records it, the job goes on
            extras[f"{name.replace(' ', '_')}_error"] = f"{type(ex).__name__}: {ex}"[:300]
        epitaph()

    def halo():
        if env.world_size > 1:
            extras["halo_exchange_us"] = round(halo_latency(env, solver, iters) * 1e6, 2)
            inline = info["transport"].endswith("inline halo")
            extras["halo_exchange_kind"] = (f"{_plane(transport)[0]}{' blocking exchange (the fused passes exchange inline)' if inline else ''}, "
                                            f"{info['tsteps']}-wide faces + corners "
                                            f"of the {shape[0]}x{shape[1]} field, process grid "
                                            f"{info['dims'][0]}x{info['dims'][1]}")
        extras["residual_l2"] = solver.residual()

    extra("halo latency", halo)
    solver.close()
    if env.is_gpu:
        torch.cuda.empty_cache()
    if env.world_size == 1:
        def self_halo():
            t, nbytes, kind = self_halo_latency(env, shape, tsteps, iters)
            extras["halo_exchange_us"] = round(t * 1e6, 2)
            extras["halo_exchange_kind"] = (f"1-rank periodic {kind} self-exchange, {tsteps}-wide faces + "
                                            f"corners of the {shape[0]}x{shape[1]} field ({nbytes} bytes)")

        extra("self halo latency", self_halo)
    # the other orientation of a non-square process grid (BASELINE names
    # "2x4"; choose_dims may pick 4x2): the same run with PY and PX swapped,
    # so both rates are on record (profiles/r03_shares.md)
    hp, hx = info["dims"]
    if env.world_size > 1 and hp != hx and args.scaling == "strong":
        def alt():
            eng3, dt3, info3 = bench_native(env, shape, args.steps, args.warmup, overlap, (hx, hp), graph,
                                            tsteps if tsteps > 1 else False, args.wg_waves, args.seg_rows,
                                            args.init, args.seed, not args.no_calibrate, transport)
            try:
                if not args.no_timed_check:
                    checked(extras, timed_check(env, eng3, args.warmup + args.steps, args.init, args.seed,
                                                "stencil_alt_dims_check"))
            finally:
                eng3.close()
            extras["stencil_alt_dims"] = f"{hx}x{hp}"
            extras["stencil_alt_dims_MLUPS"] = round(points * args.steps / dt3 / 1e6, 1)
            extras["stencil_alt_dims_overlap"] = info3["overlap"]
            if env.is_gpu:
                torch.cuda.empty_cache()

        extra("swapped process grid run", alt)
    if args.small_size:
        def small():
            s2 = (args.small_size, args.small_size)
            # 1000 sweeps of 8192^2 are 14 ms of GPU work: 100 (1.4 ms) read
            # 3-4% low, mostly the host round trip and the clock ramp around
            # so short a timed region (profiles/r04_shares.md)
            steps2 = args.small_steps or max(1000 if env.is_gpu else 100, 4 * args.steps)
            # warm-up: 15 ms of timed passes follow a phase of host work
            # (engine set-up, calibration, the headline's check); 10 warm-up
            # sweeps read 3% low against the same passes after 2 s of
            # back-to-back work at the same shader clock (profiles/r06_clock/)
            w2 = args.small_warmup if args.small_warmup > 0 else max(args.warmup, 2000 if env.is_gpu else 10)
            eng2, dt2, info2 = bench_native(env, s2, steps2, w2, overlap, dims, graph,
                                            tsteps if tsteps > 1 else False, args.wg_waves, args.seg_rows,
                                            args.init, args.seed, not args.no_calibrate, transport)
            try:
                if not args.no_timed_check:
                    checked(extras, timed_check(env, eng2, w2 + steps2, args.init, args.seed,
                                                f"stencil_{args.small_size}_check"))
            finally:
                eng2.close()
            extras[f"stencil_{args.small_size}_MLUPS"] = round(s2[0] * s2[1] * steps2 / dt2 / 1e6, 1)
            extras[f"stencil_{args.small_size}_ms_per_step"] = round(dt2 / steps2 * 1e3, 5)
            extras[f"stencil_{args.small_size}_sclk_mhz"] = info2["clock"]["sclk_mhz"]
            extras[f"stencil_{args.small_size}_pass_plan"] = f"{steps2} steps: {info2['pass_plan']}"

        extra("small-domain stencil run", small)
    if env.world_size > 1:
        def refh():
            extras.update(ref_halo(env, args.ref_n_local, args.ref_n_other, args.ref_iters, _plane(transport)[0]))
            bad = (extras["ref_halo_dim0_bad_ghosts"], extras["ref_halo_dim1_bad_ghosts"])
            if any(bad):
                raise RuntimeError(f"wrong ghost cells after an exchange (dim 0: {bad[0]}, dim 1: {bad[1]})")

        extra("reference halo benchmark", refh)

    def daxpy():
        gbps, ddt = bench_daxpy(env, args.daxpy_n, iters=20)
        extras["daxpy_GBps"] = round(gbps, 1)
        extras["daxpy_GBps_per_gpu"] = round(gbps / env.world_size, 1)
        extras["daxpy_n"] = args.daxpy_n
        extras["daxpy_ms"] = round(ddt * 1e3, 4)

    extra("daxpy", daxpy)

    def allred():
        extras.update(daxpy_allreduce(env, args.daxpy_n, iters=20, transport=_plane(transport)[0]))
        if not extras["daxpy_allsum_rel_err"] <= 1e-9:
            raise RuntimeError(f"DAXPY ALLSUM {extras['daxpy_allsum']} differs from the closed form "
                               f"{extras['daxpy_allsum_exact']} (rel err {extras['daxpy_allsum_rel_err']:.3e})")

    extra("daxpy all-reduce", allred)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=32768, help="global domain is size x size (default 32768)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong (default): the global domain is size x size for every N (the BASELINE "
                         "config); weak: size x size PER GPU, global (py*size) x (px*size)"),
    ap.add_argument("--overlap", choices=("auto", "on", "off"), default="auto",
                    help="halo exchange overlapped with the interior pass: auto = time both once at "
                         "start-up on the real links, every rank keeps the faster")
    ap.add_argument("--no-overlap", action="store_true", help="same as --overlap off")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="hipGraph replay of the fused passes (auto = off: a fused pass is >0.5 ms of "
                         "GPU work, its launches hide behind it, profiles/r01_frame.md)")
    ap.add_argument("--tblock", choices=("on", "off"), default="on",
                    help="temporal blocking: --tsteps sweeps per memory pass and per halo exchange; "
                         "bitwise the same result as single sweeps")
    ap.add_argument("--tsteps", type=int, default=0, choices=range(0, MAX_TSTEPS + 1), metavar=f"0-{MAX_TSTEPS}",
                    help=f"sweeps per fused pass with --tblock on (2-{MAX_TSTEPS}; 0 = default {DEFAULT_TSTEPS})")
    ap.add_argument("--wg-waves", type=int, default=0, choices=range(0, 9), metavar="0-8",
                    help="temporal-blocking kernel: 128-column waves per workgroup (0 = auto)")
    ap.add_argument("--seg-rows", type=int, default=0, help="temporal-blocking kernel: rows per workgroup (0 = auto)")
    ap.add_argument("--dims", type=str, default=None, help="process grid PYxPX, e.g. 4x2")
    ap.add_argument("--init", choices=("random", "analytic"), default="random",
                    help="initial field: random (default: uniform [0,1), a hash of the global lattice "
                         "point and --seed, the same for every process grid) or analytic x^3+y^2")
    ap.add_argument("--seed", type=int, default=20261017, help="random-init seed")
    ap.add_argument("--no-calibrate", action="store_true",
                    help="plan passes from the built-in cost table instead of timing each pass size "
                         "on the real share at start-up")
    ap.add_argument("--daxpy-n", type=int, default=1 << 28)
    ap.add_argument("--small-warmup", type=int, default=0,
                    help="untimed warm-up sweeps of the second stencil domain (0: max(--warmup, 2000) on the GPU, "
                         "max(--warmup, 10) on the CPU backend)")
    ap.add_argument("--small-steps", type=int, default=0,
                    help="timed steps of the second stencil domain (0: max(1000, 4 x --steps) on the GPU, "
                         "max(100, 4 x --steps) on the CPU backend)")
    ap.add_argument("--small-size", type=int, default=8192,
                    help="second stencil domain (BASELINE single-GPU config 8192^2; 0 = skip)")
    ap.add_argument("--skip-extras", action="store_true", help="headline stencil only")
    ap.add_argument("--skip-check", action="store_true", help="skip the small-domain correctness gate")
    ap.add_argument("--no-timed-check", action="store_true",
                    help="skip the check of the timed runs (their final fields against a single-sweep replay, "
                         "bitwise on the device; a mismatch exits 6)")
    ap.add_argument("--ref-n-local", type=int, default=1024,
                    help="reference halo benchmark (N>1): n_local_deriv (mpi_stencil2d_gt default 1024)")
    ap.add_argument("--ref-n-other", type=int, default=512 * 1024,
                    help="reference halo benchmark: extent of the other axis (default 512Ki: 8 MiB faces)")
    ap.add_argument("--ref-iters", type=int, default=100, help="reference halo benchmark: timed exchanges")
    ap.add_argument("--device", type=str, default=None, help="cuda|cpu (default: cuda if available)")
    ap.add_argument("--timeout", type=float, default=300.0,
                    help="hang watchdog: seconds without progress before the job fails naming the rank and "
                         "phase (GMT_TIMEOUT overrides; 0 = off)")
    ap.add_argument("--transport", choices=("auto",) + PROBE_KINDS, default="auto",
                    help="engine data plane at N > 1: rccl, ipc, or push (ipc mappings, every fused pass "
                         "stores its faces into the neighbours' ghost cells; auto: timed at start-up, see "
                         "--transport-probe)")
    ap.add_argument("--transport-probe", choices=("auto", "on", "off"), default="auto",
                    help="auto: with one rank per GPU, time RCCL and IPC (xGMI peer mappings) on the real "
                         "faces in an isolated child process group and keep the faster that passes the "
                         "bitwise gate; on: also on the CPU backend; off: RCCL")
    ap.add_argument("--probe-timeout", type=float, default=150.0, help="seconds for the transport probe")
    ap.add_argument("--probe-iters", type=int, default=50, help="timed exchanges per probed transport")
    ap.add_argument("--probe-passes", type=int, default=6,
                    help="timed fused passes per probed data plane and rep (two reps, interleaved A B C C B A)")
    ap.add_argument("--probe-port", type=int, default=0, help="the probe's rendezvous port (0: MASTER_PORT+101)")
    ap.add_argument("--probe-child", type=str, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--probe-kinds", type=str, default="", help=argparse.SUPPRESS)
    argv = sys.argv[1:] if argv is None else list(argv)
    args = ap.parse_args(argv)
    # read by the engine library when its first entry point arms the watchdog
    os.environ.setdefault("GMT_TIMEOUT", str(args.timeout))

    kinds = [] if args.probe_child else probe_kinds(args)
    probe = run_probe(args, argv, kinds) if kinds else None
    env = gdist.init(device=args.device)
    if args.gpus != env.world_size and env.rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={env.world_size}", file=sys.stderr)
    dims = tuple(int(v) for v in args.dims.lower().split("x")) if args.dims else None
    overlap_mode = "off" if args.no_overlap else args.overlap
    overlap = {"auto": "auto", "on": True, "off": False}[overlap_mode]
    gdims = dims if dims else choose_dims(env.world_size, args.size, args.size)
    if args.scaling == "weak":
        dims = gdims  # the per-GPU block stays size x size
        shape = (args.size * gdims[0], args.size * gdims[1])
    else:
        shape = (args.size, args.size)
    graph = args.graph == "on"
    tsteps = (args.tsteps or DEFAULT_TSTEPS) if args.tblock == "on" else 1
    if args.probe_child:
        probe_child(args, dims or gdims, shape, tsteps, graph)
        return
    extras = {}
    transport = args.transport
    if env.world_size > 1 and args.transport == "auto":
        mark(env, "transport choice")
        transport, cands, probe_s = agree_transport(env, probe, kinds)
        if cands is not None:
            extras["transport_candidates"] = cands
            extras["transport_probe_s"] = probe_s
    if not args.skip_check:
        mark(env, "correctness gate")
        diff = check_engine(env, dims or gdims, tsteps, graph, args.init, args.seed, transport)
        extras["check_max_diff"] = diff
        extras.update(peer_status(env, dims or gdims))
        if diff != 0.0:
            if env.rank == 0:
                print(f"bench.py: distributed result differs from the serial reference by {diff}",
                      file=sys.stderr)
            gdist.shutdown()
            sys.exit(3)
    mark(env, "headline stencil run")
    solver, dt, info = bench_native(env, shape, args.steps, args.warmup, overlap, dims, graph,
                                    tsteps if tsteps > 1 else False, args.wg_waves, args.seg_rows,
                                    args.init, args.seed, not args.no_calibrate, transport)
    points = shape[0] * shape[1]
    mlups = points * args.steps / dt / 1e6
    ms_per_step = dt / args.steps * 1e3
    py, px = info["dims"] if info.get("dims") else gdims
    extras["watchdog_timeout_s"] = watchdog_timeout("cuda" if env.is_gpu else "cpu")
    # the shader clock the timed fused passes ran at (sampled waves' s_memtime
    # over s_memrealtime; min over ranks): a run's MLUPS against its clock
    extras["timed_pass_sclk_mhz"] = info["clock"]["sclk_mhz"]
    extras["timed_pass_clock_samples"] = info["clock"]["samples"]
    if not args.no_timed_check:
        # before any extra: the halo latency and residual extras advance the field
        mark(env, "check of the timed run")
        try:
            checked(extras, timed_check(env, solver, args.warmup + args.steps, args.init, args.seed))
        except TimedCheckFailed as ex:
            extras["timed_check_error"] = str(ex)[:300]
    base = result_record(args, env, shape, mlups, ms_per_step, info, (py, px))

    def rec():
        return {**base, **extras}

    # From here on the headline is measured (and checked): every later phase
    # is an extra.  An extra that raises becomes an "<extra>_error" field; one
    # that hangs ends the job through the watchdog, which then prints this
    # line (with the extras finished so far and a "watchdog" field) and exits
    # EXTRA_HANG_EXIT (5) on every rank instead of 124 — the headline is never
    # lost to an extra, and the hang stays visible in the exit status.
    epitaph = _epitaph(env, rec)
    epitaph()
    if extras.get("timed_check_failed"):
        solver.close()
        if env.rank == 0:
            print(json.dumps(rec()), flush=True)
            print(f"bench.py: the timed field differs from its single-sweep replay: {extras['timed_check_error']}",
                  file=sys.stderr, flush=True)
        watchdog_epitaph("", TIMED_CHECK_EXIT, "cuda" if env.is_gpu else "cpu")
        gdist.shutdown()
        sys.exit(TIMED_CHECK_EXIT)
    if not args.skip_extras:
        run_extras(args, env, solver, info, shape, points, tsteps, overlap, dims, graph, transport, extras, epitaph)
    else:
        solver.close()
    mark(env, "report")
    if env.rank == 0:
        print(json.dumps(rec()), flush=True)
    # the line is out: a hang in the teardown exits quietly
    watchdog_epitaph("", 0, "cuda" if env.is_gpu else "cpu")
    failed = [k for k in extras if k.endswith("_error")]
    if failed and env.rank == 0:
        print(f"bench.py: extras failed (the headline stands): {', '.join(failed)}", file=sys.stderr)
    gdist.shutdown()
    if extras.get("timed_check_failed"):
        sys.exit(TIMED_CHECK_EXIT)


if __name__ == "__main__":
    main()
