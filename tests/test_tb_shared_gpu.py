"""Shared hand-off group launches of the temporal-blocking kernel
(csrc/kernels/jacobi5tb.hpp Sh<K>: four two-stage strips per workgroup whose
stage-1 waves read windows of one shared level-K/2 row) vs the plain fp64
PyTorch reference of k single sweeps and vs the per-strip launch, bitwise:
every K with a group kernel (12, 16, 20), widths at and around one and two
group widths (the last group shifted left to end at the rect's edge), odd
and even left offsets, Dirichlet / halo / mixed sides, exact and scaled
levels, multi-segment and multi-round launches."""
import pytest
import torch

from gpu_mpi_tests_amd import _native, ops
from gpu_mpi_tests_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
# output columns of one group (Sh<K, 4>::GOUT, Sh<K, 2>::GOUT)
GOUT = {12: 952, 16: 936, 20: 920}
GOUT2 = {12: 472, 16: 464, 20: 448}


@pytest.fixture(autouse=True, scope="module")
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.lib()


def _field(k, ny, nx, seed, xo):
    g = torch.Generator(device="cpu").manual_seed(seed)
    u = torch.rand(ny + 2 * k, xo + nx + k + 3, generator=g, dtype=torch.float64).to(DEV)
    return u, (xo, nx, k, ny)


def _run(k, u, dom, mask, shared, cpu=True, **kw):
    un = torch.full_like(u, 7.0)
    ops.jacobi5tb(k, u, un, [dom], dom, mask, shared=shared, **kw)
    torch.cuda.synchronize()
    return un.cpu() if cpu else un


def _plan(k, u, dom, mask, shared, **kw):
    return ops.jacobi5tb_plan(k, [dom], dom, mask, u.stride(0), u.shape[0], shared=shared, **kw)


@pytest.mark.parametrize("k", [12, 16, 20])
@pytest.mark.parametrize("dw", [0, 1, 2, 3, 5, None])
@pytest.mark.parametrize("mask", [0, 15, 6, 9])
def test_shared_bitwise(k, dw, mask):
    nx = 2 * GOUT[k] + 37 if dw is None else GOUT[k] + dw
    xo = 24 + (dw or 0) % 2
    u, dom = _field(k, 45, nx, seed=11 * k + nx, xo=xo)
    assert _plan(k, u, dom, mask, 1)["threads"] == 512  # the group launch runs
    got = _run(k, u, dom, mask, 1)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, [dom], dom, mask)
    assert torch.equal(got, exp), (got - exp).abs().max()
    assert torch.equal(got, _run(k, u, dom, mask, -1))


@pytest.mark.parametrize("k", [12, 20])
@pytest.mark.parametrize("seg_rows", [64, 100])
@pytest.mark.parametrize("exact", [False, True])
def test_shared_segments_exact(k, seg_rows, exact):
    """Several segments per group (warm-up rows at every segment start) and
    the exact (1/4 per level) arithmetic."""
    u, dom = _field(k, 333, 2100, seed=5 + k, xo=k + 1)
    got = _run(k, u, dom, 5, 1, seg_rows=seg_rows, exact=exact)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, [dom], dom, 5)
    assert torch.equal(got, exp), (got - exp).abs().max()


@pytest.mark.parametrize("ny,nx,seg_rows", [(4000, 9300, 64), (32768, 16384, 0)])
def test_shared_multi_round(ny, nx, seg_rows):
    """More workgroups than resident slots (several rounds; the planner's
    own segments and edges-last order on the BASELINE's 32768-row height)
    on Dirichlet fields, against the per-strip launch on the device."""
    k = 20
    u, dom = _field(k, ny, nx, seed=3, xo=k)
    p = _plan(k, u, dom, 0, 1, seg_rows=seg_rows)
    assert p["threads"] == 512 and p["workgroups"] > p["resident"], p
    a = _run(k, u, dom, 0, 1, cpu=False, seg_rows=seg_rows)
    b = _run(k, u, dom, 0, -1, cpu=False)
    assert torch.equal(a, b), int((a != b).sum())


def test_shared_not_for_narrow_or_push():
    """Rects narrower than a group and explicit workgroup shapes keep the
    per-strip launch."""
    k = 20
    u, dom = _field(k, 40, GOUT[k] - 1, seed=1, xo=k)
    assert _plan(k, u, dom, 0, 1)["threads"] == 128
    u, dom = _field(k, 40, 2000, seed=1, xo=k)
    assert _plan(k, u, dom, 0, 1, wg_waves=2)["threads"] == 256
    assert _plan(k, u, dom, 0, -1)["threads"] == 128


@pytest.mark.parametrize("ny,nx,mask,threads", [
    (32768, 32768, 0, 256),   # the BASELINE domain, Dirichlet: two-strip shared groups
    (16384, 32768, 5, 256),   # an N = 2 share (2^29 points): the same
    (16384, 16384, 0, 256),   # 2^28 points: two-strip shared groups
    (8192, 32768, 12, 256),   # the N = 4 share of a 4 x 1 grid
    (8192, 16384, 0, 128),    # 2^27 points (one round): one strip
    (8192, 8192, 0, 128),     # one-round Dirichlet: one strip
    (8192, 16384, 15, 512),   # x sides exchange halos: the shared group
    (8192, 16384, 3, 512),
    (8192, 16384, 13, 128),   # a Dirichlet x side (W: bit 0 clear)
])
def test_default_launch_shapes(ny, nx, mask, threads):
    """The K = 20 default shapes (csrc/kernels/jacobi5tb.hpp sh_launch /
    launch_tb; profiles/r06_shared/README.md), from the launch plan alone."""
    k = 20
    dom = (k, nx, k, ny)
    p = ops.jacobi5tb_plan(k, [dom], dom, mask, nx + 2 * k + 8, ny + 2 * k)
    assert p["threads"] == threads, p


@pytest.mark.parametrize("k", [12, 16, 20])
@pytest.mark.parametrize("dw", [0, 1, 3, None])
@pytest.mark.parametrize("mask", [0, 15, 6])
def test_shared_two_strip_groups_bitwise(k, dw, mask):
    """Two-strip groups (gmt_tb_opts.shared = 2: 448 output columns per
    4 waves at K = 20) against the reference and the per-strip launch."""
    nx = 3 * GOUT2[k] + 41 if dw is None else GOUT2[k] + dw
    xo = 24 + (dw or 0) % 2
    u, dom = _field(k, 45, nx, seed=13 * k + nx, xo=xo)
    assert _plan(k, u, dom, mask, 2)["threads"] == 256
    got = _run(k, u, dom, mask, 2)
    exp = torch.full(u.shape, 7.0, dtype=torch.float64)
    ref.jacobi5xk(k, u.cpu(), exp, [dom], dom, mask)
    assert torch.equal(got, exp), (got - exp).abs().max()
    assert torch.equal(got, _run(k, u, dom, mask, -1))


@pytest.mark.parametrize("mask", [0, 15])
def test_shared_two_strip_groups_multi_round(mask):
    k = 20
    u, dom = _field(k, 32768, 16384, seed=9, xo=k)
    p = _plan(k, u, dom, mask, 2)
    assert p["threads"] == 256 and p["workgroups"] > p["resident"], p
    a = _run(k, u, dom, mask, 2, cpu=False)
    b = _run(k, u, dom, mask, -1, cpu=False)
    assert torch.equal(a, b), int((a != b).sum())
