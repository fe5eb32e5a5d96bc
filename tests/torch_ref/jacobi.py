"""Distributed 2-D 5-point Jacobi solver — the flagship benchmark workload.

BASELINE.json configs "mpi_stencil2d 8192² fp64 single GPU, LDS-tiled 5-pt
Jacobi" and "mpi_stencil2d 32768² on 8 GPUs (2×4 decomp), halo
exchange/interior overlap".  (The reference itself only times halo exchanges
around a derivative stencil, mpi_stencil2d_gt.cc:511-535; Jacobi/MLUPS is the
BASELINE extension)

One step = one Jacobi sweep of the whole global domain:

    overlap=True (default, 2 streams):
      comm stream : pack W/E faces -> RCCL send/recv of all faces (N/S rows
                    zero-copy)                                   [HaloExchanger.start]
      compute     : interior core sweep (cells that need no ghost)   ┐ concurrent
      compute     : wait(RCCL) -> unpack W/E ghosts -> sweep of the  ┘
                    1-2 cell boundary frame                        [finish + rects]
    overlap=False: exchange, then one full sweep (reference-style serial).

Global boundary: Dirichlet, u = 1 on the y = -1 ghost row ("lid"), 0 on the
other three sides; interior initialised with seeded uniform random values
(synthetic data, BASELINE "random-init values").  u and un share the ghost
ring so the swap keeps the boundary condition.
"""
from __future__ import annotations

import torch

from gpu_mpi_tests_amd import ops
from gpu_mpi_tests_amd.parallel import dist as gdist
from gpu_mpi_tests_amd.parallel.decomp import CartDecomp
from .field import Field2D
from .halo import HaloExchanger


class Jacobi2D:
    def __init__(self, ny: int, nx: int, env: "gdist.DistEnv | None" = None,
                 dims: tuple[int, int] | None = None, overlap: bool = True,
                 staging: str | None = None, seed: int = 1234, rhs: bool = False,
                 lid_value: float = 1.0):
        self.env = env or gdist.get()
        e = self.env
        self.decomp = CartDecomp.create(e.world_size, e.rank, ny, nx, dims)
        self.ny_g, self.nx_g = ny, nx
        lny, lnx = self.decomp.local_shape
        dev = e.device
        self.u = Field2D(lny, lnx, 1, 1, device=dev)
        self.un = Field2D(lny, lnx, 1, 1, device=dev)
        self.overlap = overlap
        # Poisson right-hand side (optional): un = 0.25*(sum nbrs) + c1*f with c1 = -h^2/4.
        self.f = None
        self.c0, self.c1 = 0.25, 0.0
        if rhs:
            # same layout as u so absolute (y, x) storage coordinates coincide
            self.f = Field2D(lny, lnx, 1, 1, device=dev)
            h = 1.0 / (max(ny, nx) + 1)
            self.c1 = -0.25 * h * h
        self._init_values(seed, lid_value)
        if staging is None:
            staging = "host" if (e.is_gpu and e.backend == "gloo") else "none"
        group = e.host_group if staging == "host" else None
        if e.is_gpu and e.backend == "gloo" and staging != "host":
            raise ValueError("GPU ranks on a gloo process group need staging='host'")
        self.ex = {id(self.u): HaloExchanger(self.decomp, self.u, staging, group),
                   id(self.un): None}
        cs = self.ex[id(self.u)].comm_stream
        self.ex[id(self.un)] = HaloExchanger(self.decomp, self.un, staging, group, comm_stream=cs)
        self.steps_done = 0

    # ------------------------------------------------------------------ init
    def _init_values(self, seed: int, lid: float) -> None:
        g = torch.Generator(device="cpu").manual_seed(seed + self.env.rank)
        lny, lnx = self.decomp.local_shape
        vals = torch.rand(lny, lnx, generator=g, dtype=torch.float64)
        for fld in (self.u, self.un):
            fld.storage.zero_()
            fld.interior.copy_(vals)
            if self.decomp.neighbors()["north"] is None:  # global y = -1 boundary
                fld.rows(-1, 1).fill_(lid)
        if self.f is not None:
            gf = torch.Generator(device="cpu").manual_seed(seed + 7919 + self.env.rank)
            self.f.interior.copy_(torch.rand(lny, lnx, generator=gf, dtype=torch.float64))

    # ------------------------------------------------------------------ step
    def _f_view(self):
        return self.f.storage if self.f is not None else None

    def _full_region(self):
        return self.u.region()

    def _core_and_frame(self):
        """Split the interior into a core that needs no ghost cells and a
        boundary frame (<= 4 rectangles).  Core x starts at an even column so
        the core sweep keeps the 16-B vector path."""
        fu = self.u
        ny, nx = fu.ny, fu.nx
        if ny < 4 or nx < 6:
            return None, [fu.region()]
        core = fu.region(2, nx - 4, 1, ny - 2)
        frame = [
            fu.region(0, nx, 0, 1),           # first row
            fu.region(0, nx, ny - 1, 1),      # last row
            fu.region(0, 2, 1, ny - 2),       # left 2 columns
            fu.region(nx - 2, 2, 1, ny - 2),  # right 2 columns
        ]
        return core, frame

    def _sweep(self, region, resid=False):
        return ops.jacobi5(self.u.storage, self.un.storage, region, f=self._f_view(), c0=self.c0,
                           c1=self.c1, resid=resid)

    def step(self, resid: bool = False):
        """Advance one Jacobi sweep.  Returns the local sum((un-u)^2) tensor if resid."""
        ex = self.ex[id(self.u)]
        r = None
        if not ex.active:
            r = self._sweep(self._full_region(), resid)
        elif self.overlap:
            core, frame = self._core_and_frame()
            ex.start()
            if core is not None:
                r = self._sweep(core, resid)
            ex.finish()
            ops.jacobi5_rects(self.u.storage, self.un.storage, frame, f=self._f_view(), c0=self.c0,
                              c1=self.c1)
            if resid:  # frame residual (small): compute with the reference formula on views
                r = (r if r is not None else 0) + self._frame_resid(frame)
        else:
            ex.exchange()
            r = self._sweep(self._full_region(), resid)
        self.u, self.un = self.un, self.u
        self.steps_done += 1
        return r

    def _frame_resid(self, frame):
        tot = None
        for (x0, nx, y0, ny) in frame:
            if nx <= 0 or ny <= 0:
                continue
            a = self.un.storage[y0 : y0 + ny, x0 : x0 + nx]
            b = self.u.storage[y0 : y0 + ny, x0 : x0 + nx]
            d = ops.diff_sq(a, b)
            tot = d if tot is None else tot + d
        return tot if tot is not None else 0

    def run(self, n: int) -> None:
        for _ in range(n):
            self.step()

    # ------------------------------------------------------------ diagnostics
    def global_residual(self) -> float:
        """sqrt(sum over all ranks of (u_{k+1}-u_k)^2) for one extra step."""
        r = self.step(resid=True)
        v = torch.as_tensor(r, dtype=torch.float64).reshape(1).to(self.env.device)
        if self.env.world_size > 1:
            if self.env.backend == "nccl":
                torch.distributed.all_reduce(v)
            else:
                vc = v.cpu()
                torch.distributed.all_reduce(vc, group=self.env.host_group)
                v = vc
        return float(v.sqrt().item())

    def gather_global(self) -> torch.Tensor | None:
        """Assemble the global interior on rank 0 (tests / small problems only)."""
        loc = self.u.interior.contiguous().cpu()
        if self.env.world_size == 1:
            return loc
        objs = [None] * self.env.world_size
        torch.distributed.all_gather_object(objs, (self.decomp.offset, loc), group=self.env.host_group)
        if self.env.rank != 0:
            return None
        out = torch.empty(self.ny_g, self.nx_g, dtype=torch.float64)
        for (oy, ox), t in objs:
            out[oy : oy + t.shape[0], ox : ox + t.shape[1]] = t
        return out

    @property
    def points(self) -> int:
        return self.ny_g * self.nx_g

    def bytes_per_step_local(self) -> int:
        lny, lnx = self.decomp.local_shape
        per = 16 + (8 if self.f is not None else 0)
        return lny * lnx * per
