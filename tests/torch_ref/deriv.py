"""Distributed 4th-order derivative with halo exchange — torch.distributed path.

Python/torch.distributed equivalent of the reference's ``test_deriv`` and
``test_sum`` (mpi_stencil2d_gt.cc:385-649) and of the native app
``mpi_stencil2d_gt`` (csrc/apps/deriv_common.hpp).  Workload: z = x^3 + y^2 on
a 2-D field decomposed into 1-D slabs along ``dim`` (0 = contiguous x, 1 =
strided y), ghost width 2, non-periodic neighbours rank±1; after every halo
exchange the derivative d z / d(dim) is computed with the 5-point stencil
(exact for cubics, so ``err_norm`` is round-off unless the exchange is wrong).

Differences from the reference, on purpose: the fill and the error norm run
on the device (gfx950 kernels), buffers are persistent, the transport is
``torch.distributed`` (RCCL for one GPU per rank; gloo with host staging for
CPU ranks or several ranks per GPU).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from gpu_mpi_tests_amd import ops
from gpu_mpi_tests_amd.ops.reference import DERIV5
from gpu_mpi_tests_amd.parallel import dist as gdist
from gpu_mpi_tests_amd.parallel.decomp import CartDecomp
from .field import Field2D
from .halo import HaloExchanger

PI = 3.141592653598793  # the reference's constant (mpi_stencil2d_gt.cc:30)


@dataclass
class DerivResult:
    dim: int
    total_time: float  # this rank, timed iterations (s)
    err_norm: float    # this rank
    times: list = field(default_factory=list)
    bytes_per_exchange: int = 0

    @property
    def median_us(self) -> float:
        t = sorted(self.times)
        return t[len(t) // 2] * 1e6 if t else 0.0


def _sync(env):
    if env.is_gpu:
        torch.cuda.synchronize(env.device)


def run_deriv(dim: int, n_local: int, n_other: int, n_iter: int, n_warmup: int = 5,
              env: "gdist.DistEnv | None" = None, staging: str | None = None) -> DerivResult:
    """One reference ``test_deriv`` (device memory): returns this rank's times and err_norm."""
    env = env or gdist.get()
    ws, rank = env.world_size, env.rank
    nb = 2
    n_global = n_local * ws
    ln = 8.0
    delta, scale = ln / n_global, n_global / ln
    start = rank * (ln / ws)
    if dim == 0:
        decomp = CartDecomp.slab(ws, rank, n_other, n_global, axis=0)
        fld = Field2D(n_other, n_local, gy=0, gx=nb, device=env.device)
        x0, y0 = start, 0.0
    else:
        decomp = CartDecomp.slab(ws, rank, n_global, n_other, axis=1)
        fld = Field2D(n_local, n_other, gy=nb, gx=0, device=env.device)
        x0, y0 = 0.0, start
    # interior + physical-boundary ghosts (mpi_stencil2d_gt.cc:439-497)
    ops.fill_poly(fld.interior, 0, x0, delta, y0, delta)
    if dim == 0:
        if rank == 0:
            ops.fill_poly(fld.cols(-nb, nb), 0, -nb * delta, delta, 0.0, delta)
        if rank == ws - 1:
            ops.fill_poly(fld.cols(n_local, nb), 0, ln, delta, 0.0, delta)
    else:
        if rank == 0:
            ops.fill_poly(fld.rows(-nb, nb), 0, 0.0, delta, -nb * delta, delta)
        if rank == ws - 1:
            ops.fill_poly(fld.rows(n_local, nb), 0, 0.0, delta, ln, delta)
    if staging is None:
        staging = "host" if (env.is_gpu and env.backend == "gloo") else "none"
    group = env.host_group if staging == "host" else None
    ex = HaloExchanger(decomp, fld, staging, group)
    src = fld.with_ghosts if dim == 0 else fld.storage[:, fld.xo: fld.xo + fld.nx]
    res = DerivResult(dim, 0.0, 0.0, bytes_per_exchange=ex.bytes_per_exchange())
    dz = None
    for it in range(n_warmup + n_iter):
        _sync(env)
        t0 = time.perf_counter()
        ex.exchange()
        _sync(env)
        t1 = time.perf_counter()
        if it >= n_warmup:
            res.total_time += t1 - t0
            res.times.append(t1 - t0)
        # "do some calculation" between exchanges (mpi_stencil2d_gt.cc:528-534)
        dz = ops.stencil5_2d(src, dim, out=dz, scale=scale, coef=DERIV5)
        _sync(env)
    exact = torch.empty_like(dz)
    ops.fill_poly(exact, 1 if dim == 0 else 2, x0, delta, y0, delta)
    res.err_norm = ops.diff_norm(dz, exact)
    return res


def run_sum(dim: int, n_local: int, n_other: int, n_iter: int, n_warmup: int = 5,
            env: "gdist.DistEnv | None" = None) -> tuple[float, float]:
    """Reference ``test_sum``: axis-sum of a PI/world_size field to n_local values,
    then a timed in-place all-reduce.  Returns (this rank's total seconds,
    max relative error of the reduced values vs PI * n_other)."""
    env = env or gdist.get()
    ny, nx = (n_other, n_local) if dim == 0 else (n_local, n_other)
    z = torch.full((ny, nx), PI / env.world_size, dtype=torch.float64, device=env.device)
    total = 0.0
    s = None
    for it in range(n_warmup + n_iter):
        s = ops.sum_axis(z, keep_dim=0 if dim == 0 else 1)
        _sync(env)
        t0 = time.perf_counter()
        if env.world_size > 1:
            if env.backend == "nccl":
                dist.all_reduce(s)
            else:
                sc = s.cpu()
                dist.all_reduce(sc, group=env.host_group)
                s.copy_(sc)
        _sync(env)
        if it >= n_warmup:
            total += time.perf_counter() - t0
    expect = PI * n_other
    err = float(((s.cpu() - expect).abs() / expect).max())
    return total, err


def report_line(dim: int, managed: bool, buf: bool, time_sum: float, err_sum: float) -> str:
    """The reference's result line (mpi_stencil2d_gt.cc:375-383, 568-571)."""
    return (f"TEST dim:{dim}, {'managed' if managed else 'device '}, buf:{int(buf)}; "
            f"{time_sum:0.8f}, err={err_sum:0.8f}")


def reduce_sum(v: float, env) -> float:
    return gdist.reduce_sum_host(v, env)


def err_ok(err: float, n_points: int, scale: float) -> bool:
    """Round-off bound for the 5-point derivative of x^3 + y^2 (see deriv_common.hpp)."""
    return err < 1e-9 * math.sqrt(max(1, n_points)) * max(1.0, scale)
