"""Host-code sanitizers: the CPU backend, transports, halo
engine and apps built with AddressSanitizer + UBSan (``make asan-host``,
build/asan) and run under MPI.  The reference has no sanitizer coverage at
all; GPU-side ASAN is not available on the MI355X pool, so this is the
memory-safety net for the native runtime (pack/unpack indexing, IPC
mappings, persistent buffers, the watchdog thread)."""
from __future__ import annotations

import fcntl
import os
import subprocess

import pytest

from native_util import MPIRUN, ROOT, have_mpi

pytestmark = pytest.mark.skipif(not have_mpi(), reason="no mpirun")

BIN = os.path.join(ROOT, "build", "asan", "bin-host")
SAN_ENV = {
    "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=86",
    "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1:exitcode=87",
    "OMP_NUM_THREADS": "1",
}


@pytest.fixture(scope="module")
def asan_build():
    with open("/tmp/gmt_asan_build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", ROOT, f"-j{min(8, os.cpu_count() or 2)}", "asan-host"],
                       check=True, stdout=subprocess.DEVNULL)
        fcntl.flock(lk, fcntl.LOCK_UN)
    return BIN


CASES = [
    ("mpi_jacobi2d", ["50", "10", "--tblock", "--tsteps=4", "--transport=ipc", "--check"], 2),
    ("mpi_jacobi2d", ["61", "11", "--tblock", "--dims=2x2", "--periodic", "--transport=ipc", "--check"], 4),
    ("mpi_jacobi2d", ["45", "9", "--dims=1x3", "--transport=mpi-host", "--check"], 3),
    ("mpi_stencil2d_gt", ["32", "3"], 2),
    ("mpi_stencil2d_sycl", ["16", "1", "3"], 2),
    ("mpi_stencil2d_sycl_oo", ["2", "0", "3"], 2),
    ("mpi_stencil_gt", ["1"], 4),
    ("mpi_daxpy_nvtx_managed", ["--n-per-node=65536"], 2),
    ("mpi_halo_bench", ["8", "4096", "2", "--transport=ipc"], 2),
    ("mpigatherinplace", ["--n=4096"], 2),
]


@pytest.mark.parametrize("app,args,np_", CASES, ids=[f"{c[0]}-{i}" for i, c in enumerate(CASES)])
def test_app_clean_under_asan_ubsan(asan_build, app, args, np_):
    env = dict(os.environ)
    env.update(SAN_ENV)
    p = subprocess.run([MPIRUN, "-np", str(np_), os.path.join(asan_build, app), *args],
                       capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    out = p.stdout + p.stderr
    assert "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert "runtime error:" not in out, out[-4000:]
    assert p.returncode == 0, out[-4000:]
