"""Torch-facing wrappers of the libgmt gfx950 kernels.

Device tensors dispatch to the hand-written HIP kernels (``csrc/kernels``)
on the caller's current HIP stream; CPU tensors run the PyTorch reference
(``reference.py``).  There is no silent device fallback: if libgmt is
missing, device calls raise (see ``_native.lib``).

2-D fields follow ``gmt/kernels.h``: a tensor of shape ``[ny, nx]`` with
``stride(1) == 1`` (x contiguous = the reference's "dim 0"); ``stride(0)``
is the row pitch ``ld``, so views into padded / ghosted storage are accepted
without copies.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import torch

from .. import _native
from . import reference as ref
from .reference import DERIV5


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _is_dev(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


def _check2d(t: torch.Tensor, name: str):
    if t.dim() != 2 or (t.shape[1] > 1 and t.stride(1) != 1):
        raise ValueError(f"{name}: expected a 2-D tensor with unit x-stride, got {tuple(t.shape)} "
                         f"strides {t.stride()}")
    if t.dtype != torch.float64:
        raise TypeError(f"{name}: kernels are fp64 (reference precision), got {t.dtype}")


class _Coef:
    """Keeps the ctypes array alive for the duration of the (synchronous) launch call."""

    def __init__(self, coef):
        self.arr = (ctypes.c_double * 5)(*[float(c) for c in coef])
        self.ptr = ctypes.cast(self.arr, ctypes.c_void_p)


# --------------------------------------------------------------------- DAXPY
def daxpy(a: float, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """In-place ``y <- a*x + y`` (fp64, contiguous).  K1/K2."""
    if x.numel() != y.numel():
        raise ValueError("daxpy: size mismatch")
    if not (x.is_contiguous() and y.is_contiguous()):
        raise ValueError("daxpy: contiguous vectors required (incx = incy = 1)")
    if not _is_dev(y):
        return ref.daxpy(a, x, y)
    L = _native.lib()
    _native.check(L.gmt_daxpy(y.numel(), float(a), x.data_ptr(), y.data_ptr(), _stream(y)),
                  "gmt_daxpy")
    return y


# ------------------------------------------------------------ 5-tap stencils
def stencil5_1d(inp: torch.Tensor, out: torch.Tensor | None = None, scale: float = 1.0,
                coef=DERIV5) -> torch.Tensor:
    """``out[i] = scale * sum_k coef[k]*inp[i+k]``; len(out) = len(inp)-4.  K3."""
    n = inp.numel() - 4
    if not _is_dev(inp):
        r = ref.stencil5_1d(inp, scale, coef)
        if out is None:
            return r
        out.copy_(r)
        return out
    if out is None:
        out = torch.empty(n, dtype=inp.dtype, device=inp.device)
    assert inp.is_contiguous() and out.is_contiguous() and out.numel() == n
    L = _native.lib()
    cf = _Coef(coef)
    _native.check(L.gmt_stencil5_1d(n, cf.ptr, float(scale), inp.data_ptr(),
                                    out.data_ptr(), _stream(inp)), "gmt_stencil5_1d")
    return out


def stencil5_2d(inp: torch.Tensor, dim: int, out: torch.Tensor | None = None,
                scale: float = 1.0, coef=DERIV5) -> torch.Tensor:
    """5-tap stencil along ``dim`` (0 = contiguous x, 1 = strided y).  K4/K5."""
    _check2d(inp, "stencil5_2d.inp")
    ny_in, nx_in = inp.shape
    nx_out, ny_out = (nx_in - 4, ny_in) if dim == 0 else (nx_in, ny_in - 4)
    if not _is_dev(inp):
        r = ref.stencil5_2d(inp, dim, scale, coef)
        if out is None:
            return r
        out.copy_(r)
        return out
    if out is None:
        out = torch.empty(ny_out, nx_out, dtype=inp.dtype, device=inp.device)
    _check2d(out, "stencil5_2d.out")
    assert tuple(out.shape) == (ny_out, nx_out), (out.shape, ny_out, nx_out)
    L = _native.lib()
    cf = _Coef(coef)
    _native.check(L.gmt_stencil5_2d(dim, nx_out, ny_out, cf.ptr, float(scale),
                                    inp.data_ptr(), inp.stride(0), out.data_ptr(),
                                    out.stride(0), _stream(inp)), "gmt_stencil5_2d")
    return out


# ------------------------------------------------------- halo pack / unpack
def copy2d_batched(pairs: Sequence[tuple[torch.Tensor, torch.Tensor]], max_wgs: int = 0) -> None:
    """Copy each ``src`` 2-D view into ``dst`` (same shape) in ONE launch.  K6/K7/K8.
    max_wgs > 0: at most that many workgroups in a grid-stride loop (the
    exchange a band-first pass hides, Halo2D::set_pack_wgs)."""
    pairs = [(s, d) for s, d in pairs if s.numel() > 0]
    if not pairs:
        return
    if not _is_dev(pairs[0][1]):
        for s, d in pairs:
            d.copy_(s)
        return
    L = _native.lib()
    elem = pairs[0][0].element_size()
    stream = _stream(pairs[0][1])
    for i in range(0, len(pairs), _native.MAX_COPY2D):
        chunk = pairs[i : i + _native.MAX_COPY2D]
        arr = (_native.Copy2dDesc * len(chunk))()
        for k, (s, d) in enumerate(chunk):
            if s.dim() == 1:
                s = s.view(1, -1)
            if d.dim() == 1:
                d = d.view(1, -1)
            if tuple(s.shape) != tuple(d.shape):
                raise ValueError(f"copy2d: shape mismatch {tuple(s.shape)} vs {tuple(d.shape)}")
            if s.element_size() != elem or d.element_size() != elem:
                raise TypeError("copy2d: mixed element sizes")
            if (s.shape[1] > 1 and s.stride(1) != 1) or (d.shape[1] > 1 and d.stride(1) != 1):
                raise ValueError("copy2d: unit inner stride required")
            arr[k].src = s.data_ptr()
            arr[k].dst = d.data_ptr()
            arr[k].src_ld = s.stride(0)
            arr[k].dst_ld = d.stride(0)
            arr[k].width = s.shape[1]
            arr[k].height = s.shape[0]
        _native.check(L.gmt_copy2d_batched_wgs(len(chunk), ctypes.cast(arr, ctypes.c_void_p), elem,
                                               int(max_wgs), stream), "gmt_copy2d_batched_wgs")


# ---------------------------------------------------------------- reductions
def sum_axis(z: torch.Tensor, keep_dim: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """Axis sums; keep_dim 0 -> length nx (sum over y), 1 -> length ny.  K9."""
    _check2d(z, "sum_axis.z")
    ny, nx = z.shape
    n_out = nx if keep_dim == 0 else ny
    if not _is_dev(z):
        r = ref.sum_axis(z, keep_dim)
        if out is None:
            return r
        out.copy_(r)
        return out
    if out is None:
        out = torch.empty(n_out, dtype=z.dtype, device=z.device)
    L = _native.lib()
    ws = torch.empty(max(1, L.gmt_sum_axis_workspace(keep_dim, nx, ny)), dtype=torch.float64,
                     device=z.device)
    _native.check(L.gmt_sum_axis(keep_dim, nx, ny, z.data_ptr(), z.stride(0), out.data_ptr(),
                                 ws.data_ptr(), _stream(z)), "gmt_sum_axis")
    return out


def vsum(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Sum of a contiguous fp64 vector into a 1-element tensor (one HBM pass,
    deterministic order): the DAXPY partial sums, mpi_daxpy_nvtx.cc:251-268."""
    if x.dtype != torch.float64 or not x.is_contiguous():
        raise ValueError("vsum: contiguous float64 vector required")
    if out is None:
        out = torch.empty(1, dtype=torch.float64, device=x.device)
    if not _is_dev(x):
        out.copy_(x.sum().reshape(1))
        return out
    L = _native.lib()
    n = x.numel()
    ws = torch.empty(max(1, L.gmt_sum_workspace(n)), dtype=torch.float64, device=x.device)
    _native.check(L.gmt_sum(n, x.data_ptr(), out.data_ptr(), ws.data_ptr(), _stream(x)), "gmt_sum")
    return out


def abs_max(z: torch.Tensor) -> torch.Tensor:
    """0-d tensor max |z| over a 2-D (or 1-D) fp64 tensor with unit x-stride."""
    if z.dim() == 1:
        z = z.view(1, -1)
    _check2d(z, "abs_max.z")
    if not _is_dev(z):
        return z.abs().max()
    ny, nx = z.shape
    L = _native.lib()
    ws = torch.empty(max(1, L.gmt_diff_sq_workspace(nx, ny)), dtype=torch.float64, device=z.device)
    out = torch.empty((), dtype=torch.float64, device=z.device)
    _native.check(L.gmt_abs_max(nx, ny, z.data_ptr(), z.stride(0), out.data_ptr(), ws.data_ptr(), _stream(z)),
                  "gmt_abs_max")
    return out


def diff_sq(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """0-d tensor ``sum((a-b)^2)`` (un-rooted so it can be all-reduced).  K10/K12."""
    if a.dim() == 1:
        a, b = a.view(1, -1), b.view(1, -1)
    _check2d(a, "diff_sq.a")
    _check2d(b, "diff_sq.b")
    if tuple(a.shape) != tuple(b.shape):
        raise ValueError("diff_sq: shape mismatch")
    if not _is_dev(a):
        return ref.diff_sq(a, b)
    ny, nx = a.shape
    L = _native.lib()
    ws = torch.empty(max(1, L.gmt_diff_sq_workspace(nx, ny)), dtype=torch.float64, device=a.device)
    out = torch.empty((), dtype=torch.float64, device=a.device)
    _native.check(L.gmt_diff_sq(nx, ny, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                                out.data_ptr(), ws.data_ptr(), _stream(a)), "gmt_diff_sq")
    return out


def diff_bits(a: torch.Tensor, b: torch.Tensor) -> tuple[float, int]:
    """Bitwise comparison of two 2-D fp64 regions (gmt_diff_bits): (max
    |a - b| with NaN as +inf, number of elements whose 64 bits differ)."""
    if a.dim() == 1:
        a, b = a.view(1, -1), b.view(1, -1)
    _check2d(a, "diff_bits.a")
    _check2d(b, "diff_bits.b")
    if tuple(a.shape) != tuple(b.shape):
        raise ValueError("diff_bits: shape mismatch")
    if not _is_dev(a):
        ne = a.view(torch.int64) != b.view(torch.int64)
        d = (a - b).abs().nan_to_num(nan=float("inf"))[ne]
        return (float(d.max()) if d.numel() else 0.0), int(ne.sum())
    ny, nx = a.shape
    L = _native.lib()
    ws = torch.empty(max(2, 2 * L.gmt_diff_sq_workspace(nx, ny)), dtype=torch.float64, device=a.device)
    out = torch.empty(2, dtype=torch.float64, device=a.device)
    _native.check(L.gmt_diff_bits(nx, ny, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                                  out.data_ptr(), ws.data_ptr(), _stream(a)), "gmt_diff_bits")
    o = out.cpu()
    return float(o[0]), int(o[1])


def xcd_of_workgroups(n: int, device: str = "cuda") -> list[int]:
    """The XCD each workgroup of one n-workgroup launch ran on (test hook of
    gmt_push_sync's per-XCD acquire)."""
    out = torch.zeros(n, dtype=torch.int32, device=device)
    _native.check(_native.lib().gmt_xcd_of_workgroups(int(n), out.data_ptr(),
                                                      torch.cuda.current_stream(out.device).cuda_stream),
                  "gmt_xcd_of_workgroups")
    return out.cpu().tolist()


def diff_norm(a: torch.Tensor, b: torch.Tensor) -> float:
    return float(diff_sq(a, b).sqrt())


# -------------------------------------------------------------- initialisers
def fill_poly(z: torch.Tensor, mode: int, x0: float, dx: float, y0: float, dy: float) -> torch.Tensor:
    """z = x^3 + y^2 (mode 0), 3x^2 (mode 1) or 2y (mode 2) on a uniform grid."""
    if z.dim() == 1:
        z2 = z.view(1, -1)
    else:
        z2 = z
    _check2d(z2, "fill_poly.z")
    ny, nx = z2.shape
    if not _is_dev(z):
        z2.copy_(ref.poly(mode, nx, ny, x0, dx, y0, dy, dtype=z.dtype))
        return z
    L = _native.lib()
    _native.check(L.gmt_fill_poly(mode, nx, ny, float(x0), float(dx), float(y0), float(dy),
                                  z2.data_ptr(), z2.stride(0), _stream(z)), "gmt_fill_poly")
    return z


# -------------------------------------------------------------------- Jacobi
def jacobi5(u: torch.Tensor, un: torch.Tensor, region: tuple[int, int, int, int],
            f: torch.Tensor | None = None, c0: float = 0.25, c1: float = 0.0,
            resid: bool = False) -> torch.Tensor | None:
    """One 5-point Jacobi sweep of ``region = (x0, nx, y0, ny)`` (absolute
    coordinates in the 2-D storage ``u``/``un``).  Returns the 0-d tensor
    ``sum((un-u)^2)`` over the region if ``resid``."""
    _check2d(u, "jacobi5.u")
    _check2d(un, "jacobi5.un")
    x0, nx, y0, ny = (int(v) for v in region)
    if not _is_dev(u):
        r = ref.jacobi5(u, un, x0, nx, y0, ny, f, c0, c1)
        return r if resid else None
    if u.stride(0) != un.stride(0):
        raise ValueError("jacobi5: u and un must share a row pitch")
    L = _native.lib()
    r = None
    rp = 0
    if resid:
        r = torch.empty(max(2, L.gmt_jacobi_resid_workspace(nx, ny)), dtype=torch.float64,
                        device=u.device)
        rp = r.data_ptr()
    _native.check(L.gmt_jacobi5(x0, nx, y0, ny, u.data_ptr(), un.data_ptr(), u.stride(0),
                                f.data_ptr() if f is not None else 0,
                                f.stride(0) if f is not None else 0, float(c0), float(c1), rp,
                                _stream(u)), "gmt_jacobi5")
    return r[0] if resid else None


def jacobi5_rects(u: torch.Tensor, un: torch.Tensor, rects: Sequence[tuple[int, int, int, int]],
                  f: torch.Tensor | None = None, c0: float = 0.25, c1: float = 0.0) -> None:
    """Sweep up to 4 rectangles (the boundary frame of an overlapped step) in one launch."""
    rects = [tuple(int(v) for v in r) for r in rects if r[1] > 0 and r[3] > 0]
    if not rects:
        return
    if not _is_dev(u):
        for (x0, nx, y0, ny) in rects:
            ref.jacobi5(u, un, x0, nx, y0, ny, f, c0, c1)
        return
    assert len(rects) <= 4
    L = _native.lib()
    arr = (ctypes.c_int64 * (4 * len(rects)))(*[v for r in rects for v in r])
    _native.check(L.gmt_jacobi5_rects(len(rects), ctypes.cast(arr, ctypes.c_void_p),
                                      u.data_ptr(), un.data_ptr(), u.stride(0),
                                      f.data_ptr() if f is not None else 0,
                                      f.stride(0) if f is not None else 0, float(c0), float(c1),
                                      _stream(u)), "gmt_jacobi5_rects")


TB_MAX_SWEEPS = 20  # GMT_TB_MAX_SWEEPS (csrc/include/gmt/kernels.h)


def tb_supported(k: int) -> bool:
    """Sweep counts the temporal-blocking kernel is built for: 1..10 (one wave
    per strip) and even 12..20 (two waves per strip, levels split)."""
    return 1 <= k <= 10 or (10 < k <= TB_MAX_SWEEPS and k % 2 == 0)


def _check_xk_bounds(k: int, u: torch.Tensor, un: torch.Tensor, rects) -> None:
    """Host-side guard before a K-sweep launch: the kernel reads each rect plus a
    K-wide ring, so both tensors must be whole row-major fp64 arrays holding
    that ring."""
    if u.dim() != 2 or u.shape != un.shape or not (u.is_contiguous() and un.is_contiguous()):
        raise ValueError("jacobi5tb: u and un must be contiguous 2-D tensors of one shape")
    if u.dtype != torch.float64 or un.dtype != torch.float64:
        raise ValueError("jacobi5tb: fp64 only")
    rows, cols = u.shape
    for x0, nx, y0, ny in rects:
        if x0 - k < 0 or y0 - k < 0 or x0 + nx + k > cols or y0 + ny + k > rows:
            raise ValueError(f"jacobi5tb: rect {(x0, nx, y0, ny)} with its {k}-cell ring does not fit "
                             f"a {rows}x{cols} array")


def jacobi5tb(k: int, u: torch.Tensor, un: torch.Tensor, rects: Sequence[tuple[int, int, int, int]],
              dom: tuple[int, int, int, int], halo_mask: int = 0, *, wg_waves: int = 0, seg_rows: int = 0,
              exact: bool = False, push: "dict | None" = None, push_w: int = 0, shared: int = 0) -> None:
    """``k`` fused Laplace sweeps per memory pass with the temporal-blocking kernel
    (csrc/kernels/jacobi5tb.hip): ``un = J^k(u)`` on up to 8 output rects (absolute
    coordinates, each with its k-wide ring inside the array); the rest of ``un``
    is never written.  ``dom`` is the interior; bits of ``halo_mask`` (1 W, 2 E,
    4 S, 8 N) mark ghost sides owned by a neighbour (the others are fixed
    Dirichlet rings).  ``k``: see :func:`tb_supported`.  ``wg_waves``: 256-column
    strips per workgroup (0 = default), ``seg_rows``: output rows per strip (0 =
    default), ``exact``: 1/4 multiply per level instead of power-of-two scaled
    levels.  ``push`` ({direction: tensor}, directions "S" "N" "W" "E" "SW" "SE"
    "NW" "NE") with ``push_w``: the inline halo exchange (gmt_tb_opts.push) —
    the output's face cells are also stored into each tensor at the same
    coordinates (a tensor with ``un``'s row pitch).  ``shared``: the shared hand-off
    group launch (gmt_tb_opts.shared: 1 on, -1 off, 0 default = on where it applies)."""
    rects = [tuple(int(v) for v in r) for r in rects if r[1] > 0 and r[3] > 0]
    if not tb_supported(k):
        raise ValueError(f"jacobi5tb: {k} sweeps per pass is not built (1..10 or even 12..{TB_MAX_SWEEPS})")
    if not rects:
        return
    if len(rects) > 8:
        raise ValueError("jacobi5tb: at most 8 rects per launch")
    if not _is_dev(u):
        ref.jacobi5xk(k, u, un, rects, dom, halo_mask)
        return
    if u.stride(0) != un.stride(0):
        raise ValueError("jacobi5tb: u and un must share a row pitch")
    _check_xk_bounds(k, u, un, rects)
    L = _native.lib()
    arr = (ctypes.c_int64 * (4 * len(rects)))(*[v for r in rects for v in r])
    d = (ctypes.c_int64 * 4)(*[int(v) for v in dom])
    o = _native.TbOpts(int(k), int(wg_waves), int(seg_rows), int(bool(exact)))
    o.shared = int(shared)
    if push:
        order = ("S", "N", "W", "E", "SW", "SE", "NW", "NE")
        for dirn, t in push.items():
            if t.stride(0) != un.stride(0) or t.shape[0] < un.shape[0] or t.dtype != un.dtype:
                raise ValueError("jacobi5tb: a push target needs un's row pitch, rows and dtype")
            o.push[order.index(dirn)] = t.data_ptr()
        o.push_w = int(push_w)
    _native.check(L.gmt_jacobi5tb(ctypes.byref(o), len(rects), ctypes.cast(arr, ctypes.c_void_p),
                                  ctypes.cast(d, ctypes.c_void_p), int(halo_mask), u.data_ptr(),
                                  un.data_ptr(), u.stride(0), u.shape[0], _stream(u)),
                  "gmt_jacobi5tb")


def jacobi5tb_plan(k: int, rects: Sequence[tuple[int, int, int, int]], dom: tuple[int, int, int, int],
                   halo_mask: int, ld: int, nrows: int, *, wg_waves: int = 0, seg_rows: int = 0,
                   shared: int = 0) -> dict:
    """The launch :func:`jacobi5tb` would make (gmt_jacobi5tb_plan), without
    launching: workgroups, resident workgroups, threads per workgroup (512 for
    a shared hand-off group launch), interior segment rows and count, VGPRs."""
    L = _native.lib()
    rects = [tuple(int(v) for v in r) for r in rects]
    arr = (ctypes.c_int64 * (4 * len(rects)))(*[v for r in rects for v in r])
    d = (ctypes.c_int64 * 4)(*[int(v) for v in dom])
    o = _native.TbOpts(int(k), int(wg_waves), int(seg_rows), 0)
    o.shared = int(shared)
    info = (ctypes.c_int64 * 6)()
    _native.check(L.gmt_jacobi5tb_plan(ctypes.byref(o), len(rects), ctypes.cast(arr, ctypes.c_void_p),
                                       ctypes.cast(d, ctypes.c_void_p), int(halo_mask), int(ld), int(nrows),
                                       ctypes.cast(info, ctypes.c_void_p)), "gmt_jacobi5tb_plan")
    keys = ("workgroups", "resident", "threads", "seg_rows", "segments", "vgprs")
    return dict(zip(keys, (int(v) for v in info)))


def jacobi5xk(k: int, u: torch.Tensor, un: torch.Tensor, rects: Sequence[tuple[int, int, int, int]],
              dom: tuple[int, int, int, int], halo_mask: int = 0) -> None:
    """``k`` fused Laplace sweeps with the default launch: :func:`jacobi5tb`."""
    jacobi5tb(k, u, un, rects, dom, halo_mask)
