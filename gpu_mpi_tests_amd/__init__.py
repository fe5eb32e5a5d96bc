"""gpu_mpi_tests_amd — an MI355X-native GPU + distributed microbenchmark framework.

Capabilities of bd4/gpu-mpi-tests (DAXPY, distributed 5-point derivative
stencils with halo exchange, all-reduce / all-gather probes), re-designed for
AMD Instinct MI355X (gfx950): hand-written HIP kernels in ``libgmt.so``,
``torch.distributed`` over RCCL/xGMI for the Python path, and native C++ MPI
apps (``build/bin``) with the reference's executable names and report lines.

Sub-packages: ``ops`` (kernels), ``parallel`` (process groups, decomposition,
halo exchange, collectives), ``models`` (workloads: Jacobi solver, derivative
tests, distributed DAXPY), ``utils`` (timers, roctx tracing, reports).
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401,E402
