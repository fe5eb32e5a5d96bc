"""Ghosted 2-D field storage laid out for gfx950 vector access.

Reference containers: gtensor ``gtensor<double,2,space>`` of shape
``(n + 2*n_bnd, other)`` (mpi_stencil2d_gt.cc:420-425) and the SYCL
``array2d``/``span2d`` column-major wrappers (mpi_stencil2d_sycl_oo.cc:51-152,
which used 32-bit indices and leaked — SURVEY.md §5.2).

Layout here: storage is a row-major torch tensor ``[ny + 2*gy, ld]``; x is the
contiguous axis.  The interior origin column ``xo`` is rounded up to a
multiple of 8 doubles (64 B) so that every interior row starts 16-B aligned
and the kernels take their dwordx4 path; ``ld`` is padded to a multiple of 64
doubles (512 B) so each row starts on a fresh HBM burst.  All indexing in
the kernels is 64-bit.
"""
from __future__ import annotations

import torch


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


class Field2D:
    def __init__(self, ny: int, nx: int, gy: int = 1, gx: int = 1, device="cpu",
                 dtype=torch.float64, fill: float | None = 0.0, ld_align: int = 64):
        self.ny, self.nx, self.gy, self.gx = int(ny), int(nx), int(gy), int(gx)
        self.xo = _round_up(self.gx, 8) if self.gx > 0 else 0
        self.ld = _round_up(self.xo + self.nx + self.gx, ld_align)
        self.yo = self.gy
        shape = (self.ny + 2 * self.gy, self.ld)
        if fill is None:
            self.storage = torch.empty(shape, dtype=dtype, device=device)
        else:
            self.storage = torch.full(shape, float(fill), dtype=dtype, device=device)

    # -- views -------------------------------------------------------------
    @property
    def interior(self) -> torch.Tensor:
        return self.storage[self.yo : self.yo + self.ny, self.xo : self.xo + self.nx]

    @property
    def with_ghosts(self) -> torch.Tensor:
        """Interior plus the ghost frame (ghost corners included)."""
        return self.storage[:, self.xo - self.gx : self.xo + self.nx + self.gx]

    def rows(self, y0: int, n: int) -> torch.Tensor:
        """Rows [y0, y0+n) (interior-relative; may be negative into the ghosts), interior columns."""
        return self.storage[self.yo + y0 : self.yo + y0 + n, self.xo : self.xo + self.nx]

    def cols(self, x0: int, n: int) -> torch.Tensor:
        """Columns [x0, x0+n) (interior-relative), interior rows."""
        return self.storage[self.yo : self.yo + self.ny, self.xo + x0 : self.xo + x0 + n]

    def region(self, x0: int = 0, nx: int | None = None, y0: int = 0, ny: int | None = None):
        """Absolute (x0, nx, y0, ny) kernel coordinates of an interior-relative rectangle."""
        nx = self.nx - x0 if nx is None else nx
        ny = self.ny - y0 if ny is None else ny
        return (self.xo + x0, nx, self.yo + y0, ny)

    @property
    def nbytes(self) -> int:
        return self.storage.numel() * self.storage.element_size()

    def copy_from(self, other: "Field2D") -> None:
        self.storage.copy_(other.storage)
