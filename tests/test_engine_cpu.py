"""Native Jacobi engine through its C ABI (libgmt_engine.so), CPU backend.

Each case runs in a fresh interpreter: the HIP and host engine libraries share
the libgmt.so SONAME, so one process may only ever bind one backend.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import free_port
from native_util import ROOT, ensure_host_build

CODE = r"""
import json, sys
sys.path.insert(0, {root!r})
import numpy as np
from gpu_mpi_tests_amd import engine
from gpu_mpi_tests_amd.parallel import dist as gd
env = gd.init(device="cpu")
ny, nx, steps, periodic, overlap = {ny}, {nx}, {steps}, {periodic}, {overlap}
e = engine.NativeJacobi(ny, nx, env, periodic=periodic, overlap=overlap, graph=True,
                        tblock={tblock})
e.run(steps); e.synchronize()
got = e.interior()
ref = engine.serial_jacobi(ny, nx, steps, periodic)
res = e.residual()
print(json.dumps(dict(diff=float(np.abs(got - ref).max()), shape=list(got.shape),
                      transport=e.transport, overlap=e.overlap, graph=e.graph,
                      halo=e.halo_bytes, resid=res)))
e.close()
"""


def _run(tblock=False, **kw):
    ensure_host_build()
    code = CODE.format(root=ROOT, tblock=tblock, **kw)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert p.returncode == 0, p.stdout + p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("ny,nx,steps", [(1, 1, 3), (5, 7, 4), (37, 53, 9), (64, 200, 12)])
@pytest.mark.parametrize("periodic", [False, True])
def test_native_engine_matches_numpy(ny, nx, steps, periodic):
    r = _run(ny=ny, nx=nx, steps=steps, periodic=periodic, overlap=True)
    assert r["shape"] == [ny, nx]
    assert r["diff"] < 1e-13
    assert r["transport"] == "local"
    assert r["graph"] is False  # no hipGraphs on the CPU backend
    # a single rank only exchanges (with itself) when the domain wraps around
    assert (r["halo"] > 0) == periodic
    assert r["resid"] >= 0.0


def test_native_engine_serial_mode():
    r = _run(ny=40, nx=41, steps=6, periodic=True, overlap=False)
    assert r["diff"] < 1e-13 and r["overlap"] is False


@pytest.mark.parametrize("steps", [6, 7])
@pytest.mark.parametrize("periodic", [False, True])
def test_native_engine_temporal_blocking(steps, periodic):
    r = _run(ny=41, nx=66, steps=steps, periodic=periodic, overlap=True, tblock=True)
    assert r["diff"] < 1e-13


@pytest.mark.parametrize("k", [3, 4, 6, 8])
def test_native_engine_k_sweeps(k):
    r = _run(ny=41, nx=66, steps=11, periodic=True, overlap=True, tblock=k)
    assert r["diff"] < 1e-13


@pytest.mark.parametrize("transport", ["rccl", "ipc"])
@pytest.mark.parametrize("np_,ny,nx,steps,periodic,overlap,tblock,dims", [
    (2, 40, 70, 7, False, True, 0, None),
    (2, 41, 66, 9, True, True, 2, "1x2"),
    (4, 61, 75, 13, True, True, 4, "2x2"),
    (4, 60, 64, 25, False, True, 12, "2x2"),
    (3, 50, 90, 11, True, False, 8, "1x3"),
    (6, 66, 70, 10, True, True, 6, "2x3"),
    # uneven shares (156 / 157 rows): every rank must plan the same passes
    # ([20, 16, 7] for 43 sweeps) — the plan once followed each rank's own share
    (2, 313, 1695, 43, False, False, 20, "2x1"),
])
def test_native_engine_multirank(transport, np_, ny, nx, steps, periodic, overlap, tblock, dims):
    """The multi-GPU data plane of bench.py (native engine, RCCL grouped
    send/recv or the IPC transport over the socket control plane,
    temporal-blocking halos with corners, residual all-reduce) at np_ ranks
    on the CPU backend: the result equals the serial sweep."""
    ensure_host_build()
    port = str(free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(np_),
           "--master-addr", "127.0.0.1", "--master-port", port,
           os.path.join(ROOT, "tests", "engine_mp_worker.py"), str(ny), str(nx), str(steps),
           "1" if periodic else "0", "1" if overlap else "0", str(tblock)] + ([dims] if dims else [])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
                                OMP_NUM_THREADS="1", GMT_TRANSPORT=transport))
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["transport"] == f"{transport}-host"
    assert r["diff"] < 1e-13, r
    assert r["resid_same"]
    if dims:
        assert r["dims"] == [int(v) for v in dims.split("x")]


CODE_INIT = r"""
import json, sys
sys.path.insert(0, {root!r})
import numpy as np
from gpu_mpi_tests_amd import engine
from gpu_mpi_tests_amd.parallel import dist as gd
env = gd.init(device="cpu")
e = engine.NativeJacobi({ny}, {nx}, env, periodic={periodic}, overlap=True, tblock={tblock}, init={init!r},
                        seed={seed}, calibrate=True)
e.prepare({steps})  # calibration: one timed pass of every size, then the plan
plan = e.plan({steps})
e.run({steps}); e.synchronize()
ref = engine.serial_jacobi({ny}, {nx}, {steps}, {periodic}, init={init!r}, seed={seed})
print(json.dumps(dict(diff=float(np.abs(e.interior() - ref).max()), umax=e.max_abs_u0, plan=plan,
                      cost=e.pass_cost_ms(), exact=e.exact, tsteps=e.tsteps)))
e.close()
"""


@pytest.mark.parametrize("init,seed", [("random", 0), ("random", 987654321), ("analytic", 0)])
@pytest.mark.parametrize("periodic", [False, True])
def test_native_engine_init_and_calibration(init, seed, periodic):
    """Random init (gmt_fill_poly mode 5: a hash of the global lattice point)
    is bitwise the NumPy reference's; the exactness guard runs on the
    measured max|u|; a calibrated prepare() times every pass size and the
    plan covers the steps."""
    ensure_host_build()
    code = CODE_INIT.format(root=ROOT, ny=45, nx=70, steps=23, periodic=periodic, tblock=8, init=init, seed=seed)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["diff"] == 0.0, r
    assert sum(r["plan"]) == 23 and max(r["plan"]) <= 8
    assert r["cost"]["measured"] > 0 and r["cost"]["table"] > 0
    if init == "random":
        assert 0.9 < r["umax"] < 1.0  # uniform [0, 1) over ~3400 cells
    else:
        assert 1.0 < r["umax"] < 2.2  # x^3 + y^2 on the lattice, below 2 + 3h
    assert r["exact"] is False  # max|u| * 4^8 is far from overflow


def test_lattice_uniform_matches_fill_mode5():
    """ops.fill_poly mode 5 on the host backend vs the NumPy hash (the engine's
    random init): same bits, decomposition-independent."""
    ensure_host_build()
    code = r"""
import sys, ctypes, json
sys.path.insert(0, {root!r})
import numpy as np
from gpu_mpi_tests_amd import engine
lib = engine.load("cpu")
L = ctypes.CDLL(lib._name.replace("libgmt_engine.so", "libgmt.so"))
L.gmt_fill_poly.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                            ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
z = np.zeros((6, 9))
L.gmt_fill_poly(5, 9, 6, -3.0, 12345.0, 7.0, 0.0, z.ctypes.data, 9, None)
gx = np.arange(-3, 6)[None, :].repeat(6, 0); gy = np.arange(7, 13)[:, None].repeat(9, 1)
print(json.dumps(dict(same=bool((z == engine.lattice_uniform(gx, gy, 12345)).all()), lo=float(z.min()), hi=float(z.max()))))
""".format(root=ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["same"] and 0.0 <= r["lo"] and r["hi"] < 1.0


def _ipc_layout_mismatch(env):
    # rank 1 packs its faces, rank 0 moves them in place: the y faces of the
    # one-phase corner exchange then differ in size between the two sides
    os.environ["GMT_IPC_BLOCKS"] = "0" if env.rank == 1 else "1"
    from gpu_mpi_tests_amd import engine

    e = engine.NativeJacobi(64, 64, env, dims=(2, 1), periodic=True, tblock=4, transport="ipc")
    e.close()
    return "no abort"


def test_ipc_plan_refuses_mismatched_face_layouts():
    """a rank whose environment picks another face layout must not
    exchange: the IPC plan compares every message's byte count with its peer's
    during the handle exchange and aborts naming both ranks."""
    from mp_util import run_dist

    ensure_host_build()
    with pytest.raises(AssertionError) as ei:
        run_dist(_ipc_layout_mismatch, 2, free_port(), timeout=120)
    assert "disagree on the face layout" in str(ei.value), str(ei.value)[-3000:]


@pytest.mark.parametrize("ny,nx,steps,k", [(70, 300, 23, 4), (90, 600, 41, 20), (64, 520, 9, 2)])
def test_native_engine_push_one_rank_periodic(ny, nx, steps, k):
    """Inline halo exchange on one rank, periodic on both axes: every pass
    stores its faces straight into the ghost cells of its own next input
    (every neighbour is this rank), no exchange at all between passes."""
    ensure_host_build()
    code = (f"import json, sys; sys.path.insert(0, {ROOT!r}); import numpy as np;"
            "from gpu_mpi_tests_amd import engine; from gpu_mpi_tests_amd.parallel import dist as gd;"
            "env = gd.init(device='cpu');"
            f"e = engine.NativeJacobi({ny}, {nx}, env, periodic=True, overlap=False, graph=False, tblock={k},"
            " push=True, transport='local');"
            f"e.run({steps}); e.synchronize();"
            f"ref = engine.serial_jacobi({ny}, {nx}, {steps}, True);"
            "print(json.dumps(dict(push=e.push_active, diff=float(np.abs(e.interior() - ref).max()))))")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["push"] and r["diff"] == 0.0, r


@pytest.mark.parametrize("np_,ny,nx,steps,periodic,tblock,dims", [
    (2, 100, 600, 23, False, 12, "1x2"),
    (2, 140, 300, 41, True, 20, "2x1"),
    (4, 150, 700, 27, False, 4, "2x2"),
    (4, 120, 1100, 20, True, 12, "2x2"),
    (6, 190, 800, 31, True, 12, "3x2"),
    (8, 210, 1200, 45, False, 20, "2x4"),
])
def test_native_engine_push_multirank(np_, ny, nx, steps, periodic, tblock, dims):
    """Inline halo exchange at np_ ranks over the IPC transport (memfd
    mappings on the CPU backend): faces and corners go straight into the
    neighbours' ghost cells, one hand-over per pass; bitwise equal to the
    serial sweep, residual identical on every rank."""
    ensure_host_build()
    port = str(free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(np_),
           "--master-addr", "127.0.0.1", "--master-port", port,
           os.path.join(ROOT, "tests", "engine_mp_worker.py"), str(ny), str(nx), str(steps),
           "1" if periodic else "0", "0", str(tblock), dims]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
                                GMT_TRANSPORT="ipc", GMT_TEST_PUSH="1", GMT_TEST_GRAPH="0"))
    assert p.returncode == 0, p.stdout + p.stderr
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["push"], r
    assert r["diff"] == 0.0, r
    assert r["resid_same"]


def _plan(k, ks, cost, measured):
    import ctypes
    from gpu_mpi_tests_amd.engine import load
    lib = load("cpu")
    lib.gmt_engine_plan_from_costs.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                               ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    lib.gmt_engine_plan_from_costs.restype = ctypes.c_int
    c = (ctypes.c_double * (ks + 1))(*cost)
    out = (ctypes.c_int * max(1, k))()
    n = lib.gmt_engine_plan_from_costs(k, ks, c, int(measured), out, max(1, k))
    return list(out[:n])


def test_pass_plan_tie_break():
    """The pass planner's 2% handicap on measured passes shorter than the
    full K: calibration noise of ~1% must not displace full
    passes, a real 3% gain must."""
    ks = 20
    cost = [0.0] + [0.05 + 0.0150 * K for K in range(1, ks + 1)]  # ms: launch + sweeps
    # 18-sweep passes 1% cheaper per sweep than their share of a 20-sweep pass
    c18 = list(cost)
    c18[18] = cost[20] * 18 / 20 * 0.99
    assert _plan(1000, ks, c18, measured=True) == [20] * 50
    # ... and 4% cheaper: they win even with the handicap (where they fit)
    c18[18] = cost[20] * 18 / 20 * 0.96
    plan = _plan(360, ks, c18, measured=True)
    assert sum(plan) == 360 and plan.count(18) == 20
    # table costs (not measured) get no handicap: 1% is enough
    c18[18] = cost[20] * 18 / 20 * 0.99
    plan = _plan(360, ks, c18, measured=False)
    assert sum(plan) == 360 and plan.count(18) == 20
    # full passes first, the remainder largest first
    assert _plan(45, ks, cost, measured=True)[:2] == [20, 20]
