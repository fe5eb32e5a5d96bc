"""roctx ranges and the profiler capture window, for Python callers.

Same names and semantics as the native ``gmt_trace_push/pop`` and
``gmt_profiler_start/stop`` (csrc/runtime/rt_hip.cpp), which replace the
reference's NVTX ranges and cudaProfilerStart/Stop (mpi_daxpy_nvtx.cc:167-328).
Active only when a GPU is present (rocprofv3 --marker-trace picks them up);
a no-op on CPU so the host-backend engine can load in the same process.
"""
from __future__ import annotations

import contextlib

import torch

_lib = None


def _get():
    global _lib
    if _lib is None:
        if not torch.cuda.is_available():
            _lib = False
        else:
            from .. import _native

            _lib = _native.lib() if _native.available() else False
    return _lib or None


@contextlib.contextmanager
def range_ctx(name: str):
    lib = _get()
    if lib is not None:
        lib.gmt_trace_push(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.gmt_trace_pop()


def profiler_start() -> None:
    lib = _get()
    if lib is not None:
        lib.gmt_profiler_start()


def profiler_stop() -> None:
    lib = _get()
    if lib is not None:
        lib.gmt_profiler_stop()
