"""Distributed DAXPY + all-gather — torch.distributed path.

Python equivalent of ``mpi_daxpy_nvtx_{managed,unmanaged}``
(/root/reference/mpi_daxpy_nvtx.cc:85-343; native: csrc/apps/mpi_daxpy_nvtx.cpp):
n = nodes * n_per_node / world_size doubles per rank, x = (i+1)/n, y = -x,
y <- 2x + y (the gfx950 kernel), local SUM = (n+1)/2, then the two
all-gathers (x in place, y out of place) and ALLSUM = world_size*(n+1)/2.
Timed like the reference (kernel, gather, total) with roctx ranges of the
same names.  The all-gathers go through ``torch.distributed`` — RCCL over
xGMI for one GPU per rank, gloo on host copies otherwise.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

from gpu_mpi_tests_amd import ops
from gpu_mpi_tests_amd.parallel import dist as gdist
from gpu_mpi_tests_amd.utils.trace import range_ctx

MB = 1024 * 1024


@dataclass
class DaxpyDistResult:
    n: int
    nodes: int
    sum: float
    allsum: float
    t_total: float
    t_kernel: float
    t_gather: float
    transport: str

    def lines(self, rank: int, world: int) -> list[str]:
        """The reference's per-rank report lines (mpi_daxpy_nvtx.cc:268,310,333-340)."""
        return [f"{rank}/{world} SUM = {self.sum:f}", f"{rank}/{world} ALLSUM = {self.allsum:f}",
                f"{rank}/{world} TIME total  : {self.t_total:0.3f}",
                f"{rank}/{world} TIME kernel : {self.t_kernel:0.3f}",
                f"{rank}/{world} TIME barrier: {0.0:0.3f}",
                f"{rank}/{world} TIME gather : {self.t_gather:0.3f}"]


def _sync(env):
    if env.is_gpu:
        torch.cuda.synchronize(env.device)


def _all_gather(out: torch.Tensor, inp: torch.Tensor, env) -> str:
    if env.world_size == 1:
        out.copy_(inp)
        return "none"
    if env.backend == "nccl":
        dist.all_gather_into_tensor(out, inp)
        return "rccl"
    oc = out.cpu() if out.device.type != "cpu" else out
    dist.all_gather_into_tensor(oc, inp.cpu(), group=env.host_group)
    if oc is not out:
        out.copy_(oc)
    return "gloo-host"


def run(n_per_node: int = 48 * MB, env: "gdist.DistEnv | None" = None) -> DaxpyDistResult:
    env = env or gdist.get()
    ws, rank = env.world_size, env.rank
    nodes = env.node_count
    n = nodes * n_per_node // ws
    dev = env.device
    t_start = time.perf_counter()
    with range_ctx("allocateArrays"):
        x = torch.empty(n, dtype=torch.float64, device=dev)
        y = torch.empty(n, dtype=torch.float64, device=dev)
        allx = torch.empty(n * ws, dtype=torch.float64, device=dev)
        ally = torch.empty(n * ws, dtype=torch.float64, device=dev)
    with range_ctx("initializeArrays"):
        x.copy_((torch.arange(n, dtype=torch.float64, device=dev) + 1) / n)
        y.copy_(-x)
    _sync(env)
    t0 = time.perf_counter()
    with range_ctx("cublasDaxpy"):
        ops.daxpy(2.0, x, y)
        _sync(env)
    t_kernel = time.perf_counter() - t0
    with range_ctx("localSum"):
        s = float(y.sum())
    with range_ctx("copyPrepAllxInplace"):
        allx[rank * n:(rank + 1) * n].copy_(x)
    gdist.barrier(env)
    t0 = time.perf_counter()
    with range_ctx("mpiAllGather"):
        with range_ctx("x"):
            transport = _all_gather(allx, allx[rank * n:(rank + 1) * n].clone(), env)
        with range_ctx("y"):
            _all_gather(ally, y, env)
        _sync(env)
    t_gather = time.perf_counter() - t0
    with range_ctx("allSum"):
        allsum = float(ally.sum())
    t_total = time.perf_counter() - t_start
    return DaxpyDistResult(n, nodes, s, allsum, t_total, t_kernel, t_gather, transport)
