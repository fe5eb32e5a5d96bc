"""Temporal-blocking Jacobi kernel (csrc/kernels/jacobi5tb.hip)
vs the plain fp64 PyTorch reference of k single sweeps (ops/reference.py
jacobi5xk): bitwise, every ghost-side pattern, partial strips / segments, odd
right edges, 1..8 waves per workgroup, exact and scaled arithmetic, frame-rect
launches, and nothing written outside the rects."""
import pytest
import torch

from gpu_mpi_tests_amd import _native, ops
from gpu_mpi_tests_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.lib()


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(*shape, generator=g, dtype=torch.float64) * scale).to(DEV)


def _field(k, ny, nx, seed, scale=1.0):
    g, xo = k, max(8, k + (k & 1))
    u = _rand(ny + 2 * g, (xo + nx + max(9, k + 1)) // 2 * 2, seed=seed, scale=scale)
    return u, (xo, nx, g, ny)


def _check(k, u, dom, mask, rects=None, **kw):
    xo, nx, g, ny = dom
    rects = rects or [dom]
    un = torch.full_like(u, 7.0)
    ops.jacobi5tb(k, u, un, rects, dom, mask, **kw)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, rects, dom, mask)
    torch.cuda.synchronize()
    got = un.cpu()
    assert torch.equal(got, exp), (got - exp).abs().max()


@pytest.mark.parametrize("k", [2, 4, 8, 12, 14, 16])
@pytest.mark.parametrize("wg", [0, 1, 8])
@pytest.mark.parametrize("ny,nx", [(1, 2), (7, 9), (40, 126), (33, 130), (70, 515), (301, 700), (129, 1031)])
@pytest.mark.parametrize("mask", [0, 15, 6, 9])
def test_tb_bitwise(k, wg, ny, nx, mask):
    u, dom = _field(k, ny, nx, seed=81 + k)
    _check(k, u, dom, mask, wg_waves=wg)


@pytest.mark.parametrize("k", [4, 10, 12, 16])
@pytest.mark.parametrize("seg", [1, 5, 7, 13, 64, 97])
@pytest.mark.parametrize("wg", [2, 4, 5])
def test_tb_segments(k, seg, wg):
    """Segments shorter than the pipeline (warm-up and drain overlap), and
    workgroups whose last waves have no strip."""
    u, dom = _field(k, 97, 611, seed=91)
    _check(k, u, dom, 5, seg_rows=seg, wg_waves=wg)


@pytest.mark.parametrize("k", [2, 8, 14, 16])
@pytest.mark.parametrize("mask", [0, 15, 3, 12])
def test_tb_exact(k, mask):
    u, dom = _field(k, 75, 333, seed=93)
    _check(k, u, dom, mask, exact=True)


@pytest.mark.parametrize("k", [8, 16])
def test_tb_extreme_magnitudes(k):
    """Scaled levels (4^p u_p) stay bitwise for tiny normal magnitudes; the exact
    form covers magnitudes where 4^k |u| would overflow."""
    u, dom = _field(k, 50, 260, seed=95, scale=1e-300)
    _check(k, u, dom, 15)
    u, dom = _field(k, 50, 260, seed=96, scale=1e300)
    _check(k, u, dom, 15, exact=True)


@pytest.mark.parametrize("k", [4, 12, 14])
@pytest.mark.parametrize("mask", [15, 0, 5, 10])
def test_tb_frame_rects(k, mask):
    """core + up to 4 frame bands (one launch each) == one full launch; the
    frame launch is a single 4-rect call; multi-rect launches of up to 8."""
    u, dom = _field(k, 90, 400, seed=97)
    xo, nx, g, ny = dom
    full = torch.full_like(u, 7.0)
    ops.jacobi5tb(k, u, full, [dom], dom, mask)
    split = torch.full_like(u, 7.0)
    ka = k + (k & 1)
    core = (xo + ka, nx - 2 * ka, g + k, ny - 2 * k)
    ops.jacobi5tb(k, u, split, [core], dom, mask)
    frame = [(xo, nx, g, k), (xo, nx, g + ny - k, k), (xo, ka, g + k, ny - 2 * k),
             (xo + nx - ka, ka, g + k, ny - 2 * k)]
    ops.jacobi5tb(k, u, split, frame, dom, mask)
    torch.cuda.synchronize()
    assert torch.equal(split, full)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, [dom], dom, mask)
    assert torch.equal(full.cpu(), exp)
    eight = [(xo + 2 * i * 24, 24 + (i % 2), g + 3 * i, 40 - i) for i in range(8)]
    _check(k, u, dom, mask, rects=eight)
