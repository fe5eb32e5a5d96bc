"""Inline halo exchange (gmt_tb_opts.push, csrc/kernels/jacobi5tb.hpp) on the
GPU: the fused pass stores its output's face cells a second time into other
buffers, and the engine runs whole solves with it.

* kernel level: every direction's target receives exactly its face (rows,
  columns or corner of the output, at the same coordinates) and nothing else;
  the pass's own output stays bitwise equal to the fp64 reference of k single
  sweeps;
* engine level: one rank on a periodic domain (every push lands in its own
  next input) and two / four ranks sharing the GPU over IPC mappings
  (tests/test_multirank_gpu.py runs the multi-process launcher) are bitwise
  equal to the serial NumPy solve."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import free_port
from gpu_mpi_tests_amd import _native, ops
from gpu_mpi_tests_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
DIRS = ("S", "N", "W", "E", "SW", "SE", "NW", "NE")
NO_PUSH = (6, 7, 8, 9, 10, 14)  # gmt::tb::tb_push_built (csrc/include/gmt/tb_geom.h)


@pytest.fixture(autouse=True, scope="module")
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.lib()


def _face(d, dom, w):
    x0, nx, y0, ny = dom
    xs = slice(x0, x0 + w) if "W" in d else (slice(x0 + nx - w, x0 + nx) if "E" in d else slice(x0, x0 + nx))
    ys = slice(y0, y0 + w) if d.startswith("S") else (slice(y0 + ny - w, y0 + ny) if d.startswith("N")
                                                      else slice(y0, y0 + ny))
    return ys, xs


@pytest.mark.parametrize("k", [k for k in range(1, 21) if ops.tb_supported(k) and k not in NO_PUSH])
@pytest.mark.parametrize("ny,nx", [(46, 300), (130, 517), (333, 1100)])
@pytest.mark.parametrize("dirs", [DIRS, ("S", "N"), ("W", "E"), ("S", "W", "SW"), ("N", "E", "NE", "SE")])
@pytest.mark.parametrize("w", [20, 4])
def test_push_faces_kernel(k, ny, nx, dirs, w):
    if ny < 2 * w + 2:
        pytest.skip("the kernel needs two segments clear of each other's face")
    g = max(k, 1)
    xo = 24
    gen = torch.Generator(device="cpu").manual_seed(ny * 7 + nx + k)
    u = torch.rand(ny + 2 * g, xo + nx + g + 5, generator=gen, dtype=torch.float64).to(DEV)
    dom = (xo, nx, g, ny)
    un = torch.full_like(u, 7.0)
    tg = {d: torch.full_like(u, 3.0) for d in dirs}
    ops.jacobi5tb(k, u, un, [dom], dom, 15, push=tg, push_w=w)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, [dom], dom, 15)
    torch.cuda.synchronize()
    assert torch.equal(un.cpu(), exp), (un.cpu() - exp).abs().max()
    for d, t in tg.items():
        want = torch.full(u.shape, 3.0, dtype=torch.float64)
        ys, xs = _face(d, dom, w)
        want[ys, xs] = exp[ys, xs]
        got = t.cpu()
        assert torch.equal(got, want), (d, int((got != want).sum()))


@pytest.mark.parametrize("k", [12, 16, 20])
@pytest.mark.parametrize("wg", [2, 3])
@pytest.mark.parametrize("dirs", [DIRS, ("W", "E"), ("N", "E", "NE", "SE")])
def test_push_faces_kernel_multi_strip(k, wg, dirs):
    """Several two-stage strips per workgroup with stage-major waves (the
    default shape of push passes over 2^28 points, the N = 2 shares): face
    strips share their workgroup's step barriers with plain ones."""
    ny, nx, w, g, xo = 333, 1100, 20, k, 24
    gen = torch.Generator(device="cpu").manual_seed(ny + nx + k + wg)
    u = torch.rand(ny + 2 * g, xo + nx + g + 5, generator=gen, dtype=torch.float64).to(DEV)
    dom = (xo, nx, g, ny)
    un = torch.full_like(u, 7.0)
    tg = {d: torch.full_like(u, 3.0) for d in dirs}
    ops.jacobi5tb(k, u, un, [dom], dom, 15, push=tg, push_w=w, wg_waves=wg)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, [dom], dom, 15)
    torch.cuda.synchronize()
    assert torch.equal(un.cpu(), exp), (un.cpu() - exp).abs().max()
    for d, t in tg.items():
        want = torch.full(u.shape, 3.0, dtype=torch.float64)
        ys, xs = _face(d, dom, w)
        want[ys, xs] = exp[ys, xs]
        assert torch.equal(t.cpu(), want), d


def test_push_refuses_what_it_cannot_do():
    """Odd face width, several rects, a rect other than the interior, a
    domain too short for two segments, both x faces on one strip."""
    u = torch.rand(100, 400, dtype=torch.float64, device=DEV)
    un = torch.zeros_like(u)
    t = torch.zeros_like(u)
    dom = (24, 300, 20, 60)
    for kw in (dict(push_w=5), dict(push_w=0 + 66)):
        with pytest.raises(_native.NativeError):
            ops.jacobi5tb(20, u, un, [dom], dom, 15, push={"S": t}, **kw)
    with pytest.raises(_native.NativeError):
        ops.jacobi5tb(20, u, un, [(24, 100, 20, 60), (124, 200, 20, 60)], dom, 15, push={"S": t}, push_w=20)
    with pytest.raises(_native.NativeError):  # ny < 2 w + 2
        ops.jacobi5tb(20, u, un, [(24, 300, 20, 40)], (24, 300, 20, 40), 15, push={"S": t, "N": t}, push_w=20)
    with pytest.raises(_native.NativeError):  # one strip holds both x faces
        ops.jacobi5tb(20, u, un, [(24, 200, 20, 60)], (24, 200, 20, 60), 15, push={"W": t, "E": t}, push_w=20)
    for k in NO_PUSH:  # no inline-halo kernel (it would spill): gmt_jacobi5tb_push_supported
        assert not _native.lib().gmt_jacobi5tb_push_supported(k)
        with pytest.raises(_native.NativeError):
            ops.jacobi5tb(k, u, un, [dom], dom, 15, push={"S": t}, push_w=20)


@pytest.fixture(scope="module")
def env():
    from gpu_mpi_tests_amd.parallel import dist as gd

    return gd.init(device="cuda")


@pytest.mark.parametrize("ny,nx,steps,k", [(300, 700, 43, 20), (257, 1031, 29, 12), (520, 600, 17, 4)])
def test_push_engine_one_rank_periodic(env, ny, nx, steps, k):
    """The engine's inline halo on one GPU rank, periodic on both axes: the
    faces of every pass land in its own next input (no exchange between
    passes); bitwise equal to the serial solve."""
    import numpy as np

    from gpu_mpi_tests_amd import engine

    e = engine.NativeJacobi(ny, nx, env, periodic=True, overlap=False, graph=False, tblock=k, push=True,
                            transport="local", init="random", seed=5)
    try:
        assert e.push_active
        e.run(steps)
        e.synchronize()
        got = e.interior()
    finally:
        e.close()
    want = engine.serial_jacobi(ny, nx, steps, True, init="random", seed=5)
    assert np.array_equal(got, want), float(np.abs(got - want).max())


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("np_,ny,nx,steps,periodic,k,dims", [
    (2, 400, 900, 45, True, 20, "2x1"),
    (2, 300, 1200, 33, False, 12, "1x2"),
    (4, 600, 1100, 60, True, 20, "2x2"),
    (4, 500, 1300, 29, False, 4, "2x2"),
])
def test_push_engine_ranks_sharing_the_gpu(np_, ny, nx, steps, periodic, k, dims):
    """np_ ranks on cuda:0 (IPC mappings of the same device, socket control
    plane): every pass pushes its faces and corners into the neighbours'
    buffers and hands over through the flag words; bitwise equal to the
    serial solve, residual identical on every rank."""
    port = str(free_port())
    cmd = ["timeout", "-k", "10", "150", sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(np_), "--master-addr", "127.0.0.1", "--master-port", port,
           os.path.join(ROOT, "tests", "engine_mp_worker.py"), str(ny), str(nx), str(steps),
           "1" if periodic else "0", "0", str(k), dims]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=ROOT,
                       env=dict(os.environ, OMP_NUM_THREADS="1", GMT_TRANSPORT="ipc", GMT_TEST_PUSH="1",
                                GMT_TEST_GRAPH="0", GMT_TEST_DEVICE="cuda"))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["push"] and r["diff"] == 0.0 and r["resid_same"], r
