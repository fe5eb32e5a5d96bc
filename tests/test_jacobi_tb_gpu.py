"""Temporal-blocking Jacobi kernel (csrc/kernels/jacobi5tb.hip)
vs the plain fp64 PyTorch reference of k single sweeps (ops/reference.py
jacobi5xk): bitwise, every ghost-side pattern, partial strips / segments,
right edges inside a lane (widths 0-3 mod 4), one- and two-stage strips
(k <= 10 / k >= 12: levels split over two waves with an LDS hand-off),
1..8 strips per workgroup, exact and scaled arithmetic, frame-rect launches
as the engine issues them, and nothing written outside the rects."""
import pytest
import torch

from gpu_mpi_tests_amd import _native, ops
from gpu_mpi_tests_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
KS = [k for k in range(1, 25) if ops.tb_supported(k)]


@pytest.fixture(autouse=True, scope="module")
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.lib()


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g, dtype=torch.float64) * scale).to(DEV)


def _field(k, ny, nx, seed, scale=1.0, xo=None):
    g = k
    xo = max(8, k) if xo is None else xo
    u = _rand(ny + 2 * g, xo + nx + k + 3, seed=seed, scale=scale)
    return u, (xo, nx, g, ny)


def _check(k, u, dom, mask, rects=None, **kw):
    rects = rects or [dom]
    un = torch.full_like(u, 7.0)
    ops.jacobi5tb(k, u, un, rects, dom, mask, **kw)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, rects, dom, mask)
    torch.cuda.synchronize()
    got = un.cpu()
    assert torch.equal(got, exp), (got - exp).abs().max()


def test_supported_set():
    L = _native.lib()
    for k in range(0, 27):
        assert bool(L.gmt_jacobi5tb_supported(k)) == ops.tb_supported(k), k


@pytest.mark.parametrize("k", KS)
@pytest.mark.parametrize("ny,nx", [(1, 1), (7, 9), (40, 130), (33, 191), (70, 515), (129, 1031)])
@pytest.mark.parametrize("mask", [0, 15, 6, 9])
def test_tb_bitwise(k, ny, nx, mask):
    u, dom = _field(k, ny, nx, seed=81 + k)
    _check(k, u, dom, mask)


@pytest.mark.parametrize("k", [1, 5, 10, 12, 18, 20])
@pytest.mark.parametrize("nx", [140, 141, 142, 143, 300, 301, 302])
@pytest.mark.parametrize("xo", [24, 25, 26])
def test_tb_widths_and_offsets(k, nx, xo):
    """Right edges at every lane phase, odd and even left offsets (no
    alignment requirement beyond 8 B)."""
    u, dom = _field(k, 37, nx, seed=7 * k + nx, xo=xo)
    _check(k, u, dom, 10)


@pytest.mark.parametrize("k", [2, 7, 10, 14, 20])
@pytest.mark.parametrize("wg", [1, 2, 3, 4, 8])
def test_tb_workgroup_shapes(k, wg):
    """Strips per workgroup, including workgroups whose last strips are idle
    (two-stage kernels: their waves still take every step barrier)."""
    u, dom = _field(k, 61, 733, seed=90 + k)
    _check(k, u, dom, 5, wg_waves=wg)


@pytest.mark.parametrize("k", [4, 9, 12, 20])
@pytest.mark.parametrize("seg", [1, 5, 7, 13, 64, 97])
def test_tb_segments(k, seg):
    """Segments shorter than the pipeline (warm-up and drain overlap)."""
    u, dom = _field(k, 97, 611, seed=91)
    _check(k, u, dom, 5, seg_rows=seg)


@pytest.mark.parametrize("k", [2, 3, 8, 14, 20])
@pytest.mark.parametrize("mask", [0, 15, 3, 12])
def test_tb_exact(k, mask):
    u, dom = _field(k, 75, 333, seed=93)
    _check(k, u, dom, mask, exact=True)


@pytest.mark.parametrize("k", [8, 16, 20])
def test_tb_extreme_magnitudes(k):
    """Scaled levels (4^p u_p) stay bitwise for tiny normal magnitudes; the exact
    form covers magnitudes where 4^k |u| would overflow."""
    u, dom = _field(k, 50, 260, seed=95, scale=1e-300)
    _check(k, u, dom, 15)
    u, dom = _field(k, 50, 260, seed=96, scale=1e300)
    _check(k, u, dom, 15, exact=True)


def _engine_frame(k, xo, nx, g, ny, mask):
    """The engine's overlapped block pass (csrc/engine/jacobi.cpp
    enqueue_block): core inset only on halo sides, K-wide frame bands along
    the halo sides."""
    hw, he, hs, hn = mask & 1, mask & 2, mask & 4, mask & 8
    xr = xo + nx - k
    cx0, cx1 = (xo + k if hw else xo), (xr if he else xo + nx)
    cy0, cy1 = (g + k if hs else g), (g + ny - k if hn else g + ny)
    frame = []
    if hs:
        frame.append((xo, nx, g, k))
    if hn:
        frame.append((xo, nx, g + ny - k, k))
    if hw:
        frame.append((xo, k, cy0, cy1 - cy0))
    if he:
        frame.append((xr, k, cy0, cy1 - cy0))
    return (cx0, cx1 - cx0, cy0, cy1 - cy0), frame


@pytest.mark.parametrize("k", [2, 7, 12, 20])
@pytest.mark.parametrize("mask", [15, 0, 1, 2, 5, 10, 12, 3])
@pytest.mark.parametrize("ny,nx", [(90, 400), (130, 233)])
def test_tb_engine_frame(k, mask, ny, nx):
    """core + frame launches (one-strip workgroups for the frame, as the
    engine issues them) == one full launch == the reference, and nothing
    outside the interior is written."""
    u, dom = _field(k, ny, nx, seed=73 + k)
    xo, _, g, _ = dom
    full = torch.full_like(u, 7.0)
    ops.jacobi5tb(k, u, full, [dom], dom, mask)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, [dom], dom, mask)
    split = torch.full_like(u, 7.0)
    core, frame = _engine_frame(k, xo, nx, g, ny, mask)
    ops.jacobi5tb(k, u, split, [core], dom, mask)
    ops.jacobi5tb(k, u, split, frame, dom, mask, wg_waves=1)
    torch.cuda.synchronize()
    assert torch.equal(full.cpu(), exp)
    assert torch.equal(split, full)


@pytest.mark.parametrize("k", [4, 10, 16])
def test_tb_eight_rects(k):
    u, dom = _field(k, 90, 400, seed=97)
    xo, nx, g, ny = dom
    eight = [(xo + 2 * i * 24 + (i % 3), 24 + (i % 2), g + 3 * i, 40 - i) for i in range(8)]
    _check(k, u, dom, 15, rects=eight)
