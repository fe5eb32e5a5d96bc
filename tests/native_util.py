"""Helpers for running the native apps (build/bin-host = CPU backend) under MPI."""
from __future__ import annotations

import fcntl
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN_HOST = os.path.join(ROOT, "build", "bin-host")
MPIRUN = os.environ.get("GMT_MPIRUN", "/opt/conda/bin/mpirun")
_built = False


def ensure_host_build() -> None:
    """Build the CPU backend + host apps once per session (plain g++, seconds)."""
    global _built
    if _built:
        return
    jobs = str(min(8, os.cpu_count() or 2))
    # pytest-xdist workers share the tree: serialise the (idempotent) make
    with open(os.path.join("/tmp", "gmt_host_build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", ROOT, f"-j{jobs}", "host-apps"], check=True,
                       stdout=subprocess.DEVNULL)
        fcntl.flock(lk, fcntl.LOCK_UN)
    _built = True


def have_mpi() -> bool:
    return os.path.exists(MPIRUN) or shutil.which("mpirun") is not None


def run_app(name: str, *args: str, np: int | None = None, env: dict | None = None,
            timeout: float = 120.0, check: bool = True) -> subprocess.CompletedProcess:
    ensure_host_build()
    exe = os.path.join(BIN_HOST, name)
    cmd = [exe, *args] if np is None else [MPIRUN, "-np", str(np), exe, *args]
    e = dict(os.environ)
    e.setdefault("OMP_NUM_THREADS", "1")
    if env:
        e.update(env)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd="/tmp")
    if check and p.returncode != 0:
        raise AssertionError(f"{' '.join(cmd)} failed rc={p.returncode}\n{p.stdout}\n{p.stderr}")
    return p
