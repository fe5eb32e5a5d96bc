#!/usr/bin/env python3
"""Flagship benchmark: distributed 2-D 5-point Jacobi (fp64) on MI355X.

Metric (BASELINE.json): "DAXPY GB/s + 2D stencil MLUPS at 1/2/4/8 MI355X;
halo-exchange latency".  The headline ``value`` is the whole-job stencil rate
in MLUPS (million lattice-point updates per second, summed over all GPUs) on
the BASELINE multi-GPU config "mpi_stencil2d 32768² ... (2×4 decomp), halo
exchange/interior overlap".  The global domain is FIXED at 32768² for every N
(strong scaling: N = 8 is exactly the named config).  The same JSON line also
carries the single-GPU-per-rank DAXPY bandwidth (BASELINE config "daxpy
N=2^28 fp64 on one MI355X") and the measured halo-exchange latency.

One step = one full Jacobi sweep of the global domain (every point updated
once).  The native engine (C++, ``csrc/engine/jacobi.cpp``)
runs the steps in fused passes of up to 14 sweeps by default (temporal
blocking, ``--tblock on --tsteps 14``): one 14-wide halo exchange (RCCL over
xGMI on a high-priority stream, overlapped with the interior update) and one
pass of the register-pipelined kernel (``csrc/kernels/jacobi5pipe.hip``) that
reads u(t) once and writes u(t+14) once — bitwise the same result as fourteen
single sweeps, 1/14 of the HBM bytes.  The engine splits K steps into the
cheapest sequence of passes (``JacobiSolver::plan_passes``): 100 steps = 6
14-sweep passes + 2 8-sweep passes.  ``--tblock off`` runs one exchange + one
sweep per step; ``--engine torch`` runs the single-sweep algorithm through
torch.distributed P2P from Python.  Nothing is skipped inside the timed
region: K steps are K sweeps of every lattice point (an odd K ends with one single sweep).

Launch (driver contract):
    python bench.py --gpus 1 --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

DEFAULT_TSTEPS = 14  # fused sweeps per memory pass / halo exchange (native engine; profiles/r01_k14.md)

from gpu_mpi_tests_amd import ops  # noqa: E402
from gpu_mpi_tests_amd.parallel import dist as gdist  # noqa: E402
from gpu_mpi_tests_amd.parallel.decomp import choose_dims  # noqa: E402


def default_tsteps(shape, world):
    """14 sweeps per pass, 12 for per-GPU domains below 2^27 points (8192² on
    one GPU): there the 14-deep pipeline's warm-up and ghost-rule bands cost
    more than its fewer passes save (profiles/r01_8192.md)."""
    return DEFAULT_TSTEPS if shape[0] * shape[1] // max(1, world) >= (1 << 27) else 12


def _sync(env):
    if env.is_gpu:
        torch.cuda.synchronize(env.device)


def _timed(env, fn_run, fn_sync, steps, warmup):
    fn_run(warmup)
    fn_sync()
    gdist.barrier(env)
    _sync(env)
    t0 = time.perf_counter()
    fn_run(steps)
    fn_sync()
    _sync(env)
    gdist.barrier(env)
    dt = time.perf_counter() - t0
    return gdist.allreduce_max(dt, env)


def bench_native(env, shape, steps, warmup, overlap, dims, graph, variant, tblock):
    from gpu_mpi_tests_amd.engine import NativeJacobi

    eng = NativeJacobi(shape[0], shape[1], env, dims=dims, overlap=overlap, graph=graph, variant=variant,
                       tblock=tblock)
    dt = _timed(env, eng.run, eng.synchronize, steps, warmup)
    info = {"engine": "native", "graph": eng.graph, "overlap": eng.overlap, "tblock": eng.tblock,
            "overlap_tuning": eng.tuned,
            "tsteps": eng.tsteps,
            "transport": eng.transport if env.world_size > 1 else "none",
            "halo_bytes_per_rank": eng.halo_bytes, "dims": (eng.py, eng.px)}
    return eng, dt, info


def bench_torch(env, shape, steps, warmup, overlap, dims):
    from gpu_mpi_tests_amd.models.jacobi import Jacobi2D

    solver = Jacobi2D(shape[0], shape[1], env=env, dims=dims, overlap=overlap)
    dt = _timed(env, solver.run, lambda: _sync(env), steps, warmup)
    ex = solver.ex[id(solver.u)]
    info = {"engine": "torch", "graph": False, "overlap": overlap, "tblock": False,
            "transport": env.backend if env.world_size > 1 else "none",
            "halo_bytes_per_rank": ex.bytes_per_exchange() if ex.active else 0,
            "dims": (solver.decomp.py, solver.decomp.px)}
    return solver, dt, info


def halo_latency(env, solver, iters):
    """Blocking halo exchange of the current field: mean seconds (max over ranks)."""
    if env.world_size == 1:
        return None
    exch = solver.exchange if hasattr(solver, "exchange") else solver.ex[id(solver.u)].exchange
    for _ in range(5):
        exch()
    _sync(env)
    gdist.barrier(env)
    t0 = time.perf_counter()
    for _ in range(iters):
        exch()
    _sync(env)
    dt = (time.perf_counter() - t0) / iters
    return gdist.allreduce_max(dt, env)


def ref_halo(env, n_local, n_other, iters):
    """The reference's own headline measurement (mpi_stencil2d_gt test_deriv /
    test_sum: 2-deep ghost faces of n_other doubles — 8 MiB at the defaults —
    exchanged between 1-D slab neighbours, dim 0 packed, dim 1 in place, the
    derivative kernel after each exchange; then the 1024-double all-reduce),
    over RCCL on this job's GPUs.  Per-exchange median, max over ranks."""
    from gpu_mpi_tests_amd.engine import deriv_bench

    r = deriv_bench(n_local, n_other, n_iter=iters, n_warmup=5, env=env)
    out = {"ref_halo_config": f"mpi_stencil2d_gt {n_local}x{n_other} per rank, 1-D slabs, "
                              f"{iters} exchanges, rccl"}
    for d in (0, 1):
        out[f"ref_halo_dim{d}_us"] = round(gdist.allreduce_max(r[f"dim{d}"]["median_s"], env) * 1e6, 2)
        out[f"ref_halo_dim{d}_err_norm"] = gdist.allreduce_max(r[f"dim{d}"]["err_norm"], env)
    out["ref_halo_bytes_per_rank"] = int(gdist.allreduce_max(float(r["dim0"]["bytes"]), env))
    out["ref_allreduce_1024_us"] = round(gdist.allreduce_max(r["allreduce_median_s"], env) * 1e6, 2)
    return out


def bench_daxpy(env, n, iters):
    """Per-GPU DAXPY rate (each rank on its own GPU), reported as whole-job GB/s."""
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


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=32768, help="global domain is size x size (default 32768)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong (default): the global domain is size x size for every N (the BASELINE "
                         "config); weak: size x size PER GPU, global (py*size) x (px*size)"),
    ap.add_argument("--engine", choices=("native", "torch"), default="native")
    ap.add_argument("--overlap", choices=("auto", "on", "off"), default="auto",
                    help="halo exchange overlapped with the interior pass (native engine): auto = "
                         "time both once at start-up on the real links, every rank keeps the faster")
    ap.add_argument("--no-overlap", action="store_true", help="same as --overlap off")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="hipGraph replay of the fused passes (auto = off: a 12-sweep pass is "
                         ">0.5 ms of GPU work, its 2-3 launches hide, and replaying the captured "
                         "graph measured 2-6%% slower than eager launches at every domain size, "
                         "profiles/r01_frame.md)")
    ap.add_argument("--tblock", choices=("on", "off"), default="on",
                    help="temporal blocking (native engine): --tsteps sweeps per memory pass and "
                         "per halo exchange; bitwise the same result as single sweeps")
    ap.add_argument("--tsteps", type=int, default=0,
                    help="sweeps per fused pass with --tblock on (2-14; 0 = default %d)" % DEFAULT_TSTEPS)
    ap.add_argument("--dims", type=str, default=None, help="process grid PYxPX, e.g. 4x2")
    ap.add_argument("--daxpy-n", type=int, default=1 << 28)
    ap.add_argument("--skip-extras", action="store_true", help="headline stencil only")
    ap.add_argument("--ref-n-local", type=int, default=1024,
                    help="reference halo benchmark (N>1): n_local_deriv (mpi_stencil2d_gt default 1024)")
    ap.add_argument("--ref-n-other", type=int, default=512 * 1024,
                    help="reference halo benchmark: extent of the other axis (default 512Ki: 8 MiB faces)")
    ap.add_argument("--ref-iters", type=int, default=100, help="reference halo benchmark: timed exchanges")
    ap.add_argument("--variant", type=int, default=0, help="jacobi kernel variant (0 auto,1 reg,2 lds,3 scalar)")
    ap.add_argument("--device", type=str, default=None, help="cuda|cpu (default: cuda if available)")
    args = ap.parse_args(argv)

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
    engine = args.engine
    graph = args.graph == "on"
    if engine == "native":
        solver, dt, info = bench_native(env, shape, args.steps, args.warmup, overlap, dims,
                                        graph, args.variant,
                                        (args.tsteps or default_tsteps(shape, env.world_size))
                                        if args.tblock == "on" else False)
    else:
        if env.is_gpu and args.variant:
            ops.set_jacobi_variant(args.variant)
        solver, dt, info = bench_torch(env, shape, args.steps, args.warmup, overlap_mode != "off", dims)
    points = shape[0] * shape[1]
    mlups = points * args.steps / dt / 1e6
    ms_per_step = dt / args.steps * 1e3
    extras = {}
    if not args.skip_extras:
        hl = halo_latency(env, solver, iters=max(20, min(args.steps, 200)))
        extras["halo_exchange_us"] = None if hl is None else round(hl * 1e6, 2)
        resid = solver.residual() if hasattr(solver, "residual") else solver.global_residual()
        extras["residual_l2"] = resid
        if hasattr(solver, "close"):
            solver.close()
        del solver
        if env.is_gpu:
            torch.cuda.empty_cache()
        if env.world_size > 1:
            extras.update(ref_halo(env, args.ref_n_local, args.ref_n_other, args.ref_iters))
        gbps, ddt = bench_daxpy(env, args.daxpy_n, iters=20)
        extras["daxpy_GBps"] = round(gbps, 1)
        extras["daxpy_GBps_per_gpu"] = round(gbps / env.world_size, 1)
        extras["daxpy_n"] = args.daxpy_n
        extras["daxpy_ms"] = round(ddt * 1e3, 4)
    py, px = info["dims"] if info.get("dims") else gdims
    if env.rank == 0:
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
            "data": "synthetic (analytic x^3+y^2 initial field, Dirichlet boundary)",
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
                "transport": info["transport"],
                "halo_bytes_per_rank": info["halo_bytes_per_rank"],
                "device": str(env.device),
            },
            **extras,
        }
        print(json.dumps(rec), flush=True)
    gdist.shutdown()


if __name__ == "__main__":
    main()
