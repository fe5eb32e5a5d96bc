"""Plain-PyTorch fp64 reference implementations of every libgmt kernel.

These are (1) the CPU execution path of the ops (the gtensor ``host`` backend
analogue, reference ``CMakeLists.txt:59-69``) and (2) the numerics oracle the
GPU tests compare the HIP kernels against.  Summation orders match the HIP
kernels where it matters for bitwise distributed-vs-serial checks.
"""
from __future__ import annotations

import torch

# 4th-order central first-derivative coefficients (mpi_stencil2d_gt.cc:75-76).
DERIV5 = (1.0 / 12.0, -2.0 / 3.0, 0.0, 2.0 / 3.0, -1.0 / 12.0)


def daxpy(a: float, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    y.copy_(a * x + y)
    return y


def stencil5_1d(inp: torch.Tensor, scale: float = 1.0, coef=DERIV5) -> torch.Tensor:
    n = inp.numel() - 4
    out = torch.zeros(n, dtype=inp.dtype, device=inp.device)
    for k in range(5):
        out += (coef[k] * scale) * inp[k : k + n]
    return out


def stencil5_2d(inp: torch.Tensor, dim: int, scale: float = 1.0, coef=DERIV5) -> torch.Tensor:
    """dim 0 = contiguous axis (tensor dim -1), dim 1 = strided axis (tensor dim 0)."""
    ny, nx = inp.shape
    if dim == 0:
        n = nx - 4
        out = torch.zeros(ny, n, dtype=inp.dtype, device=inp.device)
        for k in range(5):
            out += (coef[k] * scale) * inp[:, k : k + n]
    else:
        n = ny - 4
        out = torch.zeros(n, nx, dtype=inp.dtype, device=inp.device)
        for k in range(5):
            out += (coef[k] * scale) * inp[k : k + n, :]
    return out


def sum_axis(z: torch.Tensor, keep_dim: int) -> torch.Tensor:
    # keep_dim 0 keeps x (sum over rows), keep_dim 1 keeps y (sum over x).
    return z.sum(dim=0) if keep_dim == 0 else z.sum(dim=1)


def diff_sq(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    d = a - b
    return (d * d).sum()


def poly(mode: int, nx: int, ny: int, x0: float, dx: float, y0: float, dy: float,
         dtype=torch.float64, device="cpu") -> torch.Tensor:
    x = x0 + torch.arange(nx, dtype=torch.float64, device=device) * dx
    y = y0 + torch.arange(ny, dtype=torch.float64, device=device) * dy
    X = x.unsqueeze(0).expand(ny, nx)
    Y = y.unsqueeze(1).expand(ny, nx)
    if mode == 0:
        v = X * X * X + Y * Y
    elif mode == 1:
        v = 3 * X * X
    elif mode == 2:
        v = 2 * Y
    elif mode == 3:
        v = X.clone()  # linear ramp (DAXPY inputs), gmt_fill_poly mode 3
    else:
        raise ValueError(f"poly: mode {mode} (0-3 here; mode 4 is the engine's integer lattice)")
    return v.to(dtype)


def jacobi5(u: torch.Tensor, un: torch.Tensor, x0: int, nx: int, y0: int, ny: int,
            f: torch.Tensor | None = None, c0: float = 0.25, c1: float = 0.0) -> torch.Tensor | None:
    """Update un[y0:y0+ny, x0:x0+nx] from u; returns sum((un-u)^2) over the region."""
    if nx <= 0 or ny <= 0:
        return torch.zeros((), dtype=u.dtype, device=u.device)
    ys, xs = slice(y0, y0 + ny), slice(x0, x0 + nx)
    w = u[ys, x0 - 1 : x0 - 1 + nx]
    e = u[ys, x0 + 1 : x0 + 1 + nx]
    n = u[y0 - 1 : y0 - 1 + ny, xs]
    s = u[y0 + 1 : y0 + 1 + ny, xs]
    o = c0 * ((w + e) + (n + s))
    if f is not None:
        o = o + c1 * f[ys, xs]
    d = o - u[ys, xs]
    un[ys, xs] = o
    return (d * d).sum()


def jacobi5xk(k: int, u: torch.Tensor, un: torch.Tensor, rects, dom, halo_mask: int = 0) -> None:
    """fp64 reference of k fused Laplace sweeps with the ghost-side rule of
    csrc/kernels/jacobi5tb.hip: a ring cell outside ``dom`` gets an
    intermediate update only if its side's bit is set in ``halo_mask``."""
    dx0, dnx, dy0, dny = dom
    dx1, dy1 = dx0 + dnx, dy0 + dny
    for (x0, nx, y0, ny) in rects:
        cur = u[y0 - k:y0 + ny + k, x0 - k:x0 + nx + k].clone()
        for p in range(1, k + 1):
            r = k - p  # ring of this level
            xs = torch.arange(x0 - r, x0 + nx + r)
            ys = torch.arange(y0 - r, y0 + ny + r)
            sl = (slice(p, cur.shape[0] - p), slice(p, cur.shape[1] - p))
            upd = 0.25 * ((cur[p:-p, p - 1:cur.shape[1] - p - 1] + cur[p:-p, p + 1:cur.shape[1] - p + 1])
                          + (cur[p - 1:cur.shape[0] - p - 1, p:-p] + cur[p + 1:cur.shape[0] - p + 1, p:-p]))
            if p == k:
                un[y0:y0 + ny, x0:x0 + nx] = upd
                break
            rx = ((xs >= dx0) & (xs < dx1)) | torch.where(xs < dx0, bool(halo_mask & 1), bool(halo_mask & 2))
            ry = ((ys >= dy0) & (ys < dy1)) | torch.where(ys < dy0, bool(halo_mask & 4), bool(halo_mask & 8))
            nxt = cur.clone()
            nxt[sl] = torch.where(ry[:, None] & rx[None, :], upd, cur[sl])
            cur = nxt


