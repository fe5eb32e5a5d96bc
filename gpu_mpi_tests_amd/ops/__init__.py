"""Compute ops: hand-written gfx950 HIP kernels (libgmt) behind torch-facing wrappers.

Kernel inventory: K1/K2 ``daxpy``; K3 ``stencil5_1d``;
K4/K5/K11 ``stencil5_2d``; K6/K7/K8 ``copy2d_batched`` (halo pack/unpack);
K9 ``sum_axis``; K10/K12 ``diff_sq``/``diff_norm``; analytic ``fill_poly``;
and the BASELINE 5-point Jacobi ``jacobi5`` / ``jacobi5_rects`` (single sweep)
and ``jacobi5tb`` (K fused sweeps per memory pass).
"""
from .kernels import (  # noqa: F401
    abs_max,
    copy2d_batched,
    daxpy,
    diff_norm,
    diff_bits,
    diff_sq,
    xcd_of_workgroups,
    fill_poly,
    jacobi5,
    jacobi5_rects,
    jacobi5xk,
    jacobi5tb,
    jacobi5tb_plan,
    tb_supported,
    stencil5_1d,
    stencil5_2d,
    sum_axis,
    vsum,
)
from .reference import DERIV5  # noqa: F401
