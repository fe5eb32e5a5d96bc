"""CMake parity (reference build: /root/reference/CMakeLists.txt:22-83): the
CMake project configures both backends and builds the CPU host backend with
every app the Makefile builds — including ``mpi_stencil2d``, the BASELINE
benchmark name — and its ctest cases pass (daxpy checksum, distributed
Jacobi vs the serial host reference through mpirun)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APPS = ["daxpy", "daxpy_nvtx", "mpi_daxpy", "mpienv", "mpigatherinplace", "mpi_daxpy_gt", "mpi_stencil_gt",
        "mpi_stencil2d_gt", "mpi_stencil2d_sycl", "mpi_stencil2d_sycl_oo", "mpi_jacobi2d", "mpi_stencil2d",
        "mpi_halo_bench", "gmt_kernel_bench", "mpi_daxpy_nvtx_managed", "mpi_daxpy_nvtx_unmanaged"]

pytestmark = pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not installed")


def _run(cmd, cwd=None, timeout=600):
    p = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, f"{' '.join(cmd)}\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    return p.stdout


def test_cmake_host_backend_builds_and_passes_ctest(tmp_path):
    b = str(tmp_path / "build")
    _run(["cmake", "-S", ROOT, "-B", b, "-DGMT_WITH_HIP=OFF"])
    _run(["cmake", "--build", b, f"-j{min(8, os.cpu_count() or 1)}"], timeout=900)
    for app in APPS:
        assert os.path.isfile(os.path.join(b, "bin-host", app)), app
    for lib in ("libgmt.so", "libgmt_ccl.so", "libgmt_engine.so"):
        assert os.path.isfile(os.path.join(b, "lib-host", lib)), lib
    out = _run(["ctest", "--output-on-failure"], cwd=b)
    assert "100% tests passed" in out


@pytest.mark.skipif(not os.path.isdir("/opt/rocm"), reason="no ROCm toolchain")
def test_cmake_configures_the_gfx950_backend(tmp_path):
    """Configure only (the kernel build is what __graft_entry__.build() does):
    HIP language, gfx950 target, RCCL and roctx found."""
    b = str(tmp_path / "build")
    _run(["cmake", "-S", ROOT, "-B", b, "-DGMT_WITH_HOST=OFF"])
    cache = open(os.path.join(b, "CMakeCache.txt")).read()
    assert "CMAKE_HIP_ARCHITECTURES:STRING=gfx950" in cache or "gfx950" in cache
    assert "GMT_RCCL:FILEPATH=" in cache
