"""ctypes binding of ``libgmt.so`` — the hand-written gfx950 kernels.

The C ABI is declared in ``csrc/include/gmt/kernels.h``; the same library is
linked by the native MPI apps (``csrc/apps``), so Python and the apps run one
kernel code path.  The library is built in-tree (``make lib`` or
``__graft_entry__.build()``) into ``gpu_mpi_tests_amd/_lib/libgmt.so``.

Policy: CPU tensors use the pure-PyTorch reference implementations in
``ops/reference.py`` (that is what the CPU test-suite exercises); device
tensors ALWAYS go through libgmt — if it is missing, ``lib()`` raises instead
of silently falling back to PyTorch.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GMT_LIB", os.path.join(_HERE, "_lib", "libgmt.so"))

_lock = threading.Lock()
_lib = None
_load_error: Exception | None = None

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_dbl = ctypes.c_double
c_vp = ctypes.c_void_p


class Copy2dDesc(ctypes.Structure):
    _fields_ = [
        ("src", c_vp),
        ("dst", c_vp),
        ("src_ld", c_i64),
        ("dst_ld", c_i64),
        ("width", c_i64),
        ("height", c_i64),
    ]


MAX_COPY2D = 8


class StageChunk(ctypes.Structure):
    """gmt_stage_chunk (csrc/include/gmt/kernels.h)."""
    _fields_ = [
        ("src", c_vp),
        ("dst", c_vp),
        ("bytes", c_i64),
        ("rows", c_i64),
        ("ld", c_i64),
        ("first", c_i64),
        ("block", c_vp),
    ]


class TbOpts(ctypes.Structure):
    """gmt_tb_opts (csrc/include/gmt/kernels.h)."""
    _fields_ = [
        ("sweeps", c_int),
        ("wg_waves", c_int),
        ("seg_rows", c_int),
        ("exact", c_int),
        ("signal_rects", c_int),
        ("signal_count", c_vp),
        ("signal", c_vp),
        ("signal_rows", c_int),
        ("reserved_cus", c_int),
        ("signal_cols", c_int),
        ("push", c_vp * 8),
        ("push_w", c_int),
        ("stop", c_vp),
        ("clock", c_vp),
        ("shared", c_int),
    ]

_SIGS = {
    "gmt_daxpy": (c_int, [c_i64, c_dbl, c_vp, c_vp, c_vp]),
    "gmt_stencil5_1d": (c_int, [c_i64, c_vp, c_dbl, c_vp, c_vp, c_vp]),
    "gmt_stencil5_2d": (c_int, [c_int, c_i64, c_i64, c_vp, c_dbl, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "gmt_copy2d_batched": (c_int, [c_int, c_vp, c_int, c_vp]),
    "gmt_copy2d_batched_wgs": (c_int, [c_int, c_vp, c_int, c_int, c_vp]),
    "gmt_sum_axis_workspace": (c_i64, [c_int, c_i64, c_i64]),
    "gmt_sum_axis": (c_int, [c_int, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "gmt_diff_sq_workspace": (c_i64, [c_i64, c_i64]),
    "gmt_sum_workspace": (c_i64, [c_i64]),
    "gmt_sum": (c_int, [c_i64, c_vp, c_vp, c_vp, c_vp]),
    "gmt_abs_max": (c_int, [c_i64, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "gmt_diff_sq": (c_int, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "gmt_fill_poly": (c_int, [c_int, c_i64, c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_vp, c_i64, c_vp]),
    "gmt_jacobi_resid_workspace": (c_i64, [c_i64, c_i64]),
    "gmt_jacobi5": (
        c_int,
        [c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_dbl, c_dbl, c_vp, c_vp],
    ),
    "gmt_jacobi5_rects": (
        c_int,
        [c_int, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_dbl, c_dbl, c_vp],
    ),
    "gmt_jacobi5tb_supported": (c_int, [c_int]),
    "gmt_jacobi5tb_push_supported": (c_int, [c_int]),
    "gmt_jacobi5tb": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_i64, c_i64, c_vp]),
    "gmt_jacobi5tb_plan": (c_int, [c_vp, c_int, c_vp, c_vp, c_int, c_i64, c_i64, c_vp]),
    "gmt_jacobi5tb_group_cols": (c_i64, [c_int, c_int]),
    "gmt_signal_wait": (c_int, [c_vp, c_vp, c_vp, c_vp]),
    "gmt_stage_copy": (c_int, [c_int, c_vp, c_vp, c_vp, ctypes.c_uint64, c_int, c_vp]),
    "gmt_stage_scatter": (c_int, [c_int, c_vp, c_int, c_vp]),
    "gmt_poly_check": (c_int, [c_i64, c_i64, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_vp, c_i64, c_vp, c_vp]),
    "gmt_add_scalar": (c_int, [c_i64, c_i64, c_dbl, c_vp, c_i64, c_vp]),
    "gmt_error_string": (ctypes.c_char_p, [c_int]),
    "gmt_device_synchronize": (c_int, []),
    "gmt_xcd_of_workgroups": (c_int, [c_int, c_vp, c_vp]),
    "gmt_diff_bits": (c_int, [c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "gmt_build_info": (ctypes.c_char_p, []),
}


class NativeError(RuntimeError):
    pass


def _load():
    global _lib, _load_error
    with _lock:
        if _lib is not None or _load_error is not None:
            return
        try:
            # torch must own the HIP runtime first (same SONAME libamdhip64.so.7):
            # importing it here guarantees libgmt binds to the already-loaded copy.
            import torch  # noqa: F401

            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
        except Exception as e:  # pragma: no cover - exercised when lib missing
            _load_error = e


def available() -> bool:
    _load()
    return _lib is not None


def lib():
    """Return the loaded library or raise loudly (never a silent fallback)."""
    _load()
    if _lib is None:
        raise NativeError(
            f"libgmt.so could not be loaded from {LIB_PATH}: {_load_error!r}. "
            "Build it with `make lib` (or python -c 'import __graft_entry__ as g; g.build()')."
        )
    return _lib


def check(err: int, what: str) -> None:
    if err != 0:
        msg = lib().gmt_error_string(err)
        raise NativeError(f"{what} failed: hip error {err} ({msg.decode() if msg else '?'})")


def build_info() -> str:
    return lib().gmt_build_info().decode()
