"""Process-group bootstrap and rank -> GPU binding (one process per GPU).

MI355X-native replacement for the reference's per-binary MPI bootstrap
(``MPI_Init/Comm_size/Comm_rank``, e.g. mpi_stencil2d_gt.cc:670-673), node
counting (``get_node_count``, mpi_daxpy_nvtx.cc:72-82) and
``set_rank_device`` (mpi_daxpy.cc:36-62 and four copies).

Differences from the reference, deliberately:
  * the device is chosen from the NODE-LOCAL rank (``LOCAL_RANK`` from
    torchrun), not the global rank, so multi-node jobs bind correctly
    (reference bug);
  * GPU oversubscription (``n_local_ranks > n_devices``) keeps the
    reference's block mapping ``device = local_rank // (n_local/n_dev)``; as
    RCCL refuses two ranks on one GPU, an oversubscribed job automatically
    runs its collectives on ``gloo`` with host-staged buffers.
"""
from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    node_count: int = 1
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    n_devices: int = 0
    ranks_per_device: int = 1
    backend: str = "none"  # "nccl" (= RCCL on ROCm), "gloo" or "none" (single process)
    pinned_cpu: int = -1   # the core this rank pinned itself to (pin_rank), -1 = not pinned
    initialized_here: bool = False
    host_group: object = None  # a gloo group for host-side control / host-staged data

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    @property
    def device_mem_bytes(self) -> int:
        if not self.is_gpu:
            return 0
        return torch.cuda.get_device_properties(self.device).total_memory

    def rank_device_line(self) -> str:
        """The reference's binding report, mpi_daxpy.cc:58-59."""
        mem = self.device_mem_bytes // max(1, self.ranks_per_device)
        return (f"RANK[{self.rank + 1}/{self.world_size}] => "
                f"DEVICE[{(self.device.index or 0) + 1 if self.is_gpu else 0}/{self.n_devices}] mem={mem}")


_ENV: DistEnv | None = None


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def select_device(local_rank: int, local_world_size: int, n_devices: int) -> tuple[int, int]:
    """Reference ``set_rank_device`` semantics on node-local indices.

    Returns (device_index, ranks_per_device).  Raises if oversubscription is
    not an exact multiple (reference prints an ERROR and exits, mpi_daxpy.cc:44-48).
    """
    if n_devices <= 0:
        return -1, 1
    if local_world_size > n_devices:
        if local_world_size % n_devices != 0:
            raise RuntimeError(
                f"ERROR: Number of ranks ({local_world_size}) not a multiple of number of GPUs "
                f"({n_devices})")
        per = local_world_size // n_devices
        return local_rank // per, per
    return local_rank, 1


def pin_rank(local_rank: int, local_world_size: int, ranks_per_device: int) -> int:
    """Pin this process to one physical core near its GPU, a distinct core
    per local rank (native gmt_rt_pin_rank, gmt/numa_bind.hpp pin_rank_core:
    the same rule as the C++ apps' set_rank_device).  Unpinned ranks showed
    a bimodal slow mode in the host-staged exchange that ``mpirun -bind-to
    core`` removed (profiles/r05_xport/README.md); the reference's Summit
    launch binds resource sets (summit/run.sh:30).  A launcher's binding is
    only narrowed.  GMT_PIN=0 turns it off.  Returns the core's first CPU or
    -1 (nothing changed)."""
    import ctypes

    from .. import _native

    L = _native.lib()
    L.gmt_rt_pin_rank.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.gmt_rt_pin_rank.restype = ctypes.c_int
    cpu = ctypes.c_int(-1)
    L.gmt_rt_pin_rank(int(local_rank), int(local_world_size), int(ranks_per_device), ctypes.byref(cpu))
    return cpu.value


def init(backend: str | None = None, device: str | None = None, timeout_s: float = 600.0) -> DistEnv:
    """Initialise (once) the process group from torchrun-style env vars.

    ``device``: "cuda" / "cpu" / None (auto: cuda if available).
    ``backend``: "nccl" / "gloo" / None (auto: nccl on GPU unless oversubscribed).
    """
    global _ENV
    if _ENV is not None:
        return _ENV
    rank = _env_int("RANK", 0)
    world = _env_int("WORLD_SIZE", 1)
    local_rank = _env_int("LOCAL_RANK", rank)
    local_world = _env_int("LOCAL_WORLD_SIZE", world)

    want_gpu = (device == "cuda") or (device is None and torch.cuda.is_available())
    n_dev = torch.cuda.device_count() if want_gpu else 0
    env = DistEnv(rank=rank, world_size=world, local_rank=local_rank,
                  local_world_size=local_world, n_devices=n_dev)
    if want_gpu and n_dev > 0:
        idx, per = select_device(local_rank, local_world, n_dev)
        torch.cuda.set_device(idx)
        env.device = torch.device("cuda", idx)
        env.ranks_per_device = per
        if world > 1:
            env.pinned_cpu = pin_rank(local_rank, local_world, per)
    else:
        env.device = torch.device("cpu")

    if world > 1:
        if backend is None:
            backend = "nccl" if (env.is_gpu and env.ranks_per_device == 1) else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = env.device  # eager RCCL communicator init
        if not dist.is_initialized():
            from ..engine import _StdoutToStderr  # RCCL's init banner stays off stdout

            with _StdoutToStderr():
                dist.init_process_group(**kw)
            env.initialized_here = True
        env.backend = backend
        env.host_group = dist.new_group(backend="gloo") if backend != "gloo" else dist.group.WORLD
        env.node_count = _node_count(env)
    else:
        env.backend = "none"
    _ENV = env
    return env


def _node_count(env: DistEnv) -> int:
    """Reference get_node_count (MPI_Comm_split_type SHARED): count distinct hosts."""
    names = [None] * env.world_size
    dist.all_gather_object(names, socket.gethostname(), group=env.host_group)
    return max(1, len(set(names)))


def get() -> DistEnv:
    return _ENV if _ENV is not None else init()


def barrier(env: DistEnv | None = None) -> None:
    env = env or get()
    if env.world_size > 1:
        if env.backend == "nccl":
            dist.barrier(device_ids=[env.device.index])
        else:
            dist.barrier()
    if env.is_gpu:
        torch.cuda.synchronize(env.device)


def allreduce_max(value: float, env: DistEnv | None = None) -> float:
    env = env or get()
    if env.world_size == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=env.host_group)
    return float(t.item())


def reduce_sum_host(value: float, env: DistEnv | None = None) -> float:
    """Reference MPI_Reduce(SUM -> 0) of a host scalar (mpi_stencil2d_gt.cc:563,566)."""
    env = env or get()
    if env.world_size == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=env.host_group)
    return float(t.item())


def shutdown() -> None:
    global _ENV
    if _ENV is not None and _ENV.initialized_here and dist.is_initialized():
        dist.destroy_process_group()
    _ENV = None
