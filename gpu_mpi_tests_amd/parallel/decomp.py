"""Domain decomposition: 1-D slabs (reference parity) and 2-D Cartesian.

Reference: 1-D slab decomposition along dim 0 or dim 1 with non-periodic
rank±1 neighbours (mpi_stencil2d_gt.cc:401-415, mpi_stencil_gt.cc:147-148,
neighbour logic :91-107).  The 2-D ``PxQ`` Cartesian decomposition is the
BASELINE extension ("32768² on 8 GPUs (2×4 decomp)").

Axis naming follows ``gmt/kernels.h``: x = contiguous axis (reference dim 0),
y = strided axis (reference dim 1).  Ranks are laid out row-major over the
process grid: ``rank = cy * px + cx``.

MI355X note: the 8 GPUs of a node are fully connected by xGMI (every pair has
a direct link), so any 2-D process grid gives each rank <= 4 neighbours on 4
distinct links; the factorisation is therefore chosen for *message shape*,
not topology: y-faces (whole rows) are contiguous and go zero-copy, x-faces
(columns) need a pack kernel, so splits go preferentially along y.
"""
from __future__ import annotations

from dataclasses import dataclass


def _split(n: int, parts: int, idx: int) -> tuple[int, int]:
    """Balanced block split: returns (offset, length) of block ``idx``."""
    base, rem = divmod(n, parts)
    off = idx * base + min(idx, rem)
    return off, base + (1 if idx < rem else 0)


def choose_dims(world_size: int, ny: int, nx: int, x_face_penalty: float = 1.5) -> tuple[int, int]:
    """Pick (py, px) with py*px == world_size minimising the weighted halo
    volume per rank; strided x-faces cost ``x_face_penalty`` x a row face."""
    best = None
    for px in range(1, world_size + 1):
        if world_size % px:
            continue
        py = world_size // px
        ly, lx = ny / py, nx / px
        cost = (2 * lx if py > 1 else 0) + (x_face_penalty * 2 * ly if px > 1 else 0)
        key = (cost, -py)
        if best is None or key < best[0]:
            best = (key, (py, px))
    return best[1]


@dataclass
class CartDecomp:
    """A 2-D Cartesian decomposition of a global ``ny x nx`` domain."""

    world_size: int
    rank: int
    ny: int
    nx: int
    py: int
    px: int

    @classmethod
    def create(cls, world_size: int, rank: int, ny: int, nx: int,
               dims: tuple[int, int] | None = None) -> "CartDecomp":
        if dims is None:
            dims = choose_dims(world_size, ny, nx)
        py, px = dims
        if py * px != world_size:
            raise ValueError(f"process grid {py}x{px} != world size {world_size}")
        if ny < py or nx < px:
            raise ValueError(f"domain {ny}x{nx} too small for process grid {py}x{px}")
        return cls(world_size, rank, ny, nx, py, px)

    @classmethod
    def slab(cls, world_size: int, rank: int, ny: int, nx: int, axis: int) -> "CartDecomp":
        """Reference 1-D slab along ``axis`` (0 = x / dim 0, 1 = y / dim 1)."""
        return cls.create(world_size, rank, ny, nx, (1, world_size) if axis == 0 else (world_size, 1))

    @property
    def coords(self) -> tuple[int, int]:
        return divmod(self.rank, self.px)  # (cy, cx)

    def rank_of(self, cy: int, cx: int) -> int | None:
        if 0 <= cy < self.py and 0 <= cx < self.px:
            return cy * self.px + cx
        return None  # non-periodic (reference: rank 0 / N-1 have no outer neighbour)

    @property
    def local_y(self) -> tuple[int, int]:
        return _split(self.ny, self.py, self.coords[0])

    @property
    def local_x(self) -> tuple[int, int]:
        return _split(self.nx, self.px, self.coords[1])

    @property
    def local_shape(self) -> tuple[int, int]:
        return self.local_y[1], self.local_x[1]

    @property
    def offset(self) -> tuple[int, int]:
        return self.local_y[0], self.local_x[0]

    def neighbors(self) -> dict[str, int | None]:
        cy, cx = self.coords
        return {
            "north": self.rank_of(cy - 1, cx),  # y - 1
            "south": self.rank_of(cy + 1, cx),  # y + 1
            "west": self.rank_of(cy, cx - 1),   # x - 1
            "east": self.rank_of(cy, cx + 1),   # x + 1
        }

    def has_neighbors(self) -> bool:
        return any(v is not None for v in self.neighbors().values())

    def describe(self) -> str:
        return f"{self.py}x{self.px}"
