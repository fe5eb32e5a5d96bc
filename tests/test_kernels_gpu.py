"""Numerics of every hand-written HIP kernel vs a plain PyTorch fp64 reference.

GPU-only (``-m gpu``).  Sizes include odd extents, non-multiples of 64/512,
unaligned views (scalar fallback paths) and multi-block tails.
"""
import ctypes
import os

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
    _native.lib()  # must be the native path — fail loudly otherwise


def _rand(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.rand(*shape, generator=g, dtype=torch.float64).to(DEV)


@pytest.mark.parametrize("n", [1, 2, 7, 1023, 1024, 2048 * 3 + 5, 1 << 20])
def test_daxpy(n):
    x, y = _rand(n, seed=1), _rand(n, seed=2)
    exp = 2.0 * x + y
    ops.daxpy(2.0, x, y)
    torch.cuda.synchronize()
    assert torch.equal(y, exp)


def test_daxpy_unaligned():
    x, y = _rand(1001, seed=3), _rand(1001, seed=4)
    xs, ys = x[1:], y[1:]  # 8-B aligned only -> scalar kernel
    exp = 3.5 * xs + ys  # kernel contracts to one FMA: compare to 1 ulp-ish
    ops.daxpy(3.5, xs, ys)
    torch.testing.assert_close(ys, exp, rtol=1e-15, atol=1e-15)


def test_daxpy_reference_closed_form():
    # daxpy.cu:55-87: x = i+1, y = -(i+1), a = 2 -> SUM = n(n+1)/2 = 524800
    x = torch.arange(1, 1025, dtype=torch.float64, device=DEV)
    y = -x.clone()
    ops.daxpy(2.0, x, y)
    assert float(y.sum()) == 524800.0


@pytest.mark.parametrize("n", [1, 5, 513, 65536, 65536 * 3 + 17])
def test_stencil5_1d(n):
    inp = _rand(n + 4, seed=5)
    out = ops.stencil5_1d(inp, scale=3.0)
    exp = ref.stencil5_1d(inp.cpu(), 3.0).to(DEV)
    torch.testing.assert_close(out, exp, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("dim", [0, 1])
@pytest.mark.parametrize("ny,nx", [(1, 9), (7, 13), (33, 1030), (130, 516), (64, 2049)])
def test_stencil5_2d(dim, ny, nx):
    z = _rand(ny + (4 if dim == 1 else 0), nx + (4 if dim == 0 else 0), seed=6)
    out = ops.stencil5_2d(z, dim, scale=2.0)
    exp = ref.stencil5_2d(z.cpu(), dim, 2.0).to(DEV)
    torch.testing.assert_close(out, exp, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("ny,nx", [(1, 1), (1, 130), (5, 255), (8, 257), (127, 300), (129, 1031), (300, 640)])
def test_stencil5_dim1_dma_pipeline(ny, nx):
    """dim 1 through the LDS-DMA pipeline (stencil5.hip d1): segment tails,
    partial strips, odd widths (8-B edge stores), taps across segments."""
    z = _rand(ny + 4, nx, seed=16)
    out = ops.stencil5_2d(z, 1, scale=3.0)
    exp = ref.stencil5_2d(z.cpu(), 1, 3.0).to(DEV)
    torch.testing.assert_close(out, exp, rtol=1e-13, atol=1e-13)


def test_variant_bench_check():
    """The A/B variants kept out of libgmt (csrc/bench/variant_bench.hip) still
    agree with the production kernels they were measured against."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "bench", "variant_bench")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (make sweep / __graft_entry__.build())")
    p = subprocess.run([exe, "--check"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "variant_bench OK" in p.stdout, p.stdout + p.stderr


@pytest.mark.parametrize("dim", [0, 1])
def test_stencil5_2d_strided_views(dim):
    big = _rand(100, 700, seed=7)
    inp = big[3:3 + 40 + (4 if dim == 1 else 0), 2:2 + 300 + (4 if dim == 0 else 0)]
    outbig = torch.zeros(60, 800, dtype=torch.float64, device=DEV)
    out = outbig[5:45, 10:310]
    ops.stencil5_2d(inp, dim, out=out, scale=1.5)
    exp = ref.stencil5_2d(inp.cpu(), dim, 1.5).to(DEV)
    torch.testing.assert_close(out, exp, rtol=1e-13, atol=1e-13)
    # untouched outside the view
    assert float(outbig[:5].abs().sum()) == 0.0


def test_stencil_exact_for_cubic():
    # 4th-order central difference is exact for x^3
    n, dx = 4096, 1e-3
    z = torch.empty(16, n + 4, dtype=torch.float64, device=DEV)
    ops.fill_poly(z, 0, -2 * dx, dx, 0.0, 0.1)
    dz = ops.stencil5_2d(z, 0, scale=1.0 / dx)
    exact = torch.empty_like(dz)
    ops.fill_poly(exact, 1, 0.0, dx, 0.0, 0.1)
    assert ops.diff_norm(dz, exact) < 1e-7


@pytest.mark.parametrize("elem", [torch.float64, torch.float32])
def test_copy2d_batched(elem):
    src = torch.arange(50 * 40, dtype=elem, device=DEV).view(50, 40)
    bufs = [torch.zeros(50, 2, dtype=elem, device=DEV), torch.zeros(50, 1, dtype=elem, device=DEV),
            torch.zeros(3, 40, dtype=elem, device=DEV), torch.zeros(7, 33, dtype=elem, device=DEV)]
    views = [src[:, 2:4], src[:, 39:40], src[10:13, :], src[1:8, 3:36]]
    ops.copy2d_batched(list(zip(views, bufs)))
    for v, b in zip(views, bufs):
        assert torch.equal(v, b)
    # unpack back into a different array
    dst = torch.zeros_like(src)
    ops.copy2d_batched([(b, dst[:, 2:4]) for b in bufs[:1]] + [(bufs[2], dst[10:13, :])])
    assert torch.equal(dst[:, 2:4], src[:, 2:4]) and torch.equal(dst[10:13], src[10:13])


@pytest.mark.parametrize("max_wgs", [1, 3, 128])
@pytest.mark.parametrize("elem", [torch.float64, torch.float32])
def test_copy2d_batched_few_workgroups(elem, max_wgs):
    """The grid-stride form (few resident workgroups, 4 loads in flight per
    lane) moves exactly what the full-grid form moves: faces of every width
    class, a descriptor boundary inside one lane's 4-element batch."""
    src = torch.arange(300 * 70, dtype=elem, device=DEV).view(300, 70)
    views = [src[:, 2:22], src[:, 69:70], src[10:13, :], src[1:280, 3:36], src[5:6, 0:70]]
    bufs = [torch.full(v.shape, -1, dtype=elem, device=DEV) for v in views]
    ops.copy2d_batched(list(zip(views, bufs)), max_wgs=max_wgs)
    for v, b in zip(views, bufs):
        assert torch.equal(v, b)
    dst = torch.zeros_like(src)
    ops.copy2d_batched([(bufs[0], dst[:, 2:22]), (bufs[3], dst[1:280, 3:36])], max_wgs=max_wgs)
    assert torch.equal(dst[:, 2:22], src[:, 2:22]) and torch.equal(dst[1:280, 3:36], src[1:280, 3:36])


def test_copy2d_many_descriptors():
    src = _rand(64, 64, seed=8)
    pairs = [(src[i : i + 1, :], torch.empty(1, 64, dtype=torch.float64, device=DEV)) for i in range(11)]
    ops.copy2d_batched(pairs)
    for s, d in pairs:
        assert torch.equal(s, d)


@pytest.mark.parametrize("keep", [0, 1])
@pytest.mark.parametrize("ny,nx", [(1, 1), (3, 5), (1000, 1024), (1024, 9000), (77, 4097)])
def test_sum_axis(keep, ny, nx):
    z = _rand(ny, nx, seed=9)
    out = ops.sum_axis(z, keep)
    exp = ref.sum_axis(z.cpu(), keep).to(DEV)
    torch.testing.assert_close(out, exp, rtol=1e-12, atol=1e-12)


def test_sum_axis_reference_allreduce_value():
    # test_sum: fill PI/world (world=1) -> each sum = PI * extent (mpi_stencil2d_gt.cc:598-611)
    z = torch.full((2048, 1024), 3.141592653589793, dtype=torch.float64, device=DEV)
    out = ops.sum_axis(z, 0)
    torch.testing.assert_close(out, torch.full((1024,), 3.141592653589793 * 2048, dtype=torch.float64,
                                               device=DEV), rtol=1e-13, atol=0)


@pytest.mark.parametrize("ny,nx", [(1, 1), (5, 7), (300, 4100), (2, 100000)])
def test_diff_sq(ny, nx):
    a, b = _rand(ny, nx, seed=10), _rand(ny, nx, seed=11)
    got = float(ops.diff_sq(a, b))
    exp = float(ref.diff_sq(a.cpu(), b.cpu()))
    assert abs(got - exp) <= 1e-12 * max(1.0, exp)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_fill_poly(mode):
    z = torch.empty(37, 129, dtype=torch.float64, device=DEV)
    ops.fill_poly(z, mode, -0.3, 0.01, 0.2, 0.02)
    exp = ref.poly(mode, 129, 37, -0.3, 0.01, 0.2, 0.02).to(DEV)
    torch.testing.assert_close(z, exp, rtol=1e-14, atol=1e-14)


@pytest.mark.parametrize("ny,nx", [(1, 2), (3, 7), (33, 513), (64, 1024), (100, 1030)])
def test_jacobi5(ny, nx):
    u = _rand(ny + 2, nx + 16, seed=12)
    f = _rand(ny + 2, nx + 16, seed=13)
    for ff, c1 in ((None, 0.0), (f, -0.01)):
        un = torch.zeros_like(u)
        un_ref = torch.zeros(u.shape, dtype=torch.float64)
        r = ops.jacobi5(u, un, (8, nx, 1, ny), f=ff, c1=c1, resid=True)
        r_ref = ref.jacobi5(u.cpu(), un_ref, 8, nx, 1, ny, ff.cpu() if ff is not None else None, 0.25, c1)
        torch.testing.assert_close(un.cpu(), un_ref, rtol=1e-14, atol=1e-14)
        assert abs(float(r) - float(r_ref)) <= 1e-11 * max(1.0, float(r_ref))


@pytest.mark.parametrize("n", [1, 5, 4097, 1 << 20, (1 << 20) + 3])
def test_daxpy_sizes(n):
    x, y = _rand(n, seed=31), _rand(n, seed=32)
    exp = 2.0 * x + y
    ops.daxpy(2.0, x, y)
    torch.cuda.synchronize()
    assert torch.equal(y, exp)


def test_jacobi5_large_residual_two_level_reduction():
    """>1024 per-block partials: the deterministic two-level reduction."""
    ny, nx = 2000, 4000
    u = _rand(ny + 2, nx + 16, seed=41)
    un = torch.zeros_like(u)
    r = ops.jacobi5(u, un, (8, nx, 1, ny), resid=True)
    un_ref = torch.zeros(u.shape, dtype=torch.float64)
    r_ref = ref.jacobi5(u.cpu(), un_ref, 8, nx, 1, ny, None, 0.25, 0.0)
    torch.testing.assert_close(un.cpu(), un_ref, rtol=1e-14, atol=1e-14)
    assert abs(float(r) - float(r_ref)) <= 1e-10 * float(r_ref)
    r2 = ops.jacobi5(u, un, (8, nx, 1, ny), resid=True)
    assert float(r2) == float(r)  # deterministic order


def test_jacobi5_odd_origin_scalar_path():
    u = _rand(20, 40, seed=14)
    un, un_ref = torch.zeros_like(u), torch.zeros(20, 40, dtype=torch.float64)
    ops.jacobi5(u, un, (3, 31, 2, 15))
    ref.jacobi5(u.cpu(), un_ref, 3, 31, 2, 15)
    torch.testing.assert_close(un.cpu(), un_ref, rtol=1e-14, atol=1e-14)


def test_jacobi5_rects_frame():
    u = _rand(34, 80, seed=15)
    un, un_ref = torch.zeros_like(u), torch.zeros(34, 80, dtype=torch.float64)
    rects = [(8, 64, 1, 1), (8, 64, 32, 1), (8, 2, 2, 30), (70, 2, 2, 30)]
    ops.jacobi5_rects(u, un, rects)
    for r in rects:
        ref.jacobi5(u.cpu(), un_ref, *r)
    torch.testing.assert_close(un.cpu(), un_ref, rtol=1e-14, atol=1e-14)


def test_jacobi_model_single_gpu_matches_cpu():
    from torch_ref.jacobi import Jacobi2D
    from gpu_mpi_tests_amd.parallel import dist as gdist

    env_gpu = gdist.DistEnv(device=torch.device("cuda", 0), n_devices=1)
    env_cpu = gdist.DistEnv(device=torch.device("cpu"))
    a = Jacobi2D(70, 90, env=env_gpu)
    b = Jacobi2D(70, 90, env=env_cpu)
    for _ in range(7):
        a.step()
        b.step()
    torch.testing.assert_close(a.u.interior.cpu(), b.u.interior, rtol=1e-13, atol=1e-13)


def test_stream_semantics():
    """Kernels run on the caller's current stream."""
    s = torch.cuda.Stream()
    x, y = _rand(1 << 20, seed=16), _rand(1 << 20, seed=17)
    exp = 2.0 * x + y
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        ops.daxpy(2.0, x, y)
    s.synchronize()
    assert torch.equal(y, exp)


@pytest.mark.parametrize("n", [1, 2, 3, 255, 512, 513, 4097, 1 << 20, (1 << 22) + 7])
def test_vsum_matches_fp64_reference(n):
    """gmt_sum (the DAXPY partial sums) vs a plain PyTorch fp64 sum."""
    x = torch.rand(n, dtype=torch.float64, device=DEV) - 0.25
    got = float(ops.vsum(x))
    ref = float(x.double().cpu().sum())
    assert abs(got - ref) <= 1e-12 * max(1.0, float(x.abs().sum()))
    # unaligned start: the scalar path
    if n > 1:
        got2 = float(ops.vsum(x[1:]))
        assert abs(got2 - float(x[1:].cpu().sum())) <= 1e-12 * max(1.0, float(x.abs().sum()))


@pytest.mark.parametrize("ny,nx", [(1, 1), (3, 7), (257, 4099), (1000, 1024)])
def test_abs_max_matches_reference(ny, nx):
    z = torch.randn(ny, nx + 3, dtype=torch.float64, device=DEV)[:, 1:nx + 1]
    assert float(ops.abs_max(z)) == float(z.abs().max())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("rows,cols,chunk", [(2, 1000, 1 << 10), (20, 333, 4096), (3, 7, 8)])
def test_stage_gather_scatter_field_blocks(rows, cols, chunk):
    """mpi-host's in-place staging (csrc/kernels/stage.hip): a strided halo
    face gathered chunk by chunk straight out of the field into page-locked
    memory (with the per-chunk flags), then scattered back out of it into
    another block — bitwise against the packed face."""
    L = _native.lib()
    ld = rows + 37
    field = _rand(cols, ld, seed=rows)            # column-major: `cols` columns of ld doubles
    face = field[:, 5:5 + rows]                   # rows x cols block, pitch ld
    n = rows * cols
    stage = torch.zeros(n, dtype=torch.float64).pin_memory()
    nchunk = (n * 8 + chunk - 1) // chunk
    descs = (_native.StageChunk * nchunk)()
    for k in range(nchunk):
        off = k * chunk
        descs[k] = _native.StageChunk(None, stage.data_ptr() + off, min(chunk, n * 8 - off), rows, ld, off // 8,
                                      face.data_ptr())
    table = torch.empty(ctypes.sizeof(descs), dtype=torch.uint8, device=DEV)
    table.copy_(torch.frombuffer(bytearray(descs), dtype=torch.uint8))
    counters = torch.zeros(nchunk, dtype=torch.int32, device=DEV)
    flags = torch.zeros(nchunk, dtype=torch.int64).pin_memory()
    _native.check(L.gmt_stage_copy(nchunk, table.data_ptr(), counters.data_ptr(), flags.data_ptr(), 7, 4, _stream()),
                  "stage_copy")
    torch.cuda.synchronize()
    packed = face.contiguous().reshape(-1).cpu()   # packed column by column: rows per column contiguous
    assert torch.equal(stage, packed)
    assert (flags == 7).all()
    # again with more workgroups than a chunk has 16-B pieces (empty slices),
    # the arrival counters back at zero
    assert (counters == 0).all()
    stage.zero_()
    _native.check(L.gmt_stage_copy(nchunk, table.data_ptr(), counters.data_ptr(), flags.data_ptr(), 8, 300, _stream()),
                  "stage_copy")
    torch.cuda.synchronize()
    assert torch.equal(stage, packed) and (flags == 8).all() and (counters == 0).all()
    # scatter into another field's block
    out = torch.full_like(field, -1.0)
    dst = out[:, 9:9 + rows]
    for k in range(nchunk):
        off = k * chunk
        descs[k] = _native.StageChunk(stage.data_ptr() + off, None, min(chunk, n * 8 - off), rows, ld, off // 8,
                                      dst.data_ptr())
    table.copy_(torch.frombuffer(bytearray(descs), dtype=torch.uint8))
    _native.check(L.gmt_stage_scatter(nchunk, table.data_ptr(), 3, _stream()), "stage_scatter")
    torch.cuda.synchronize()
    assert torch.equal(out[:, 9:9 + rows].cpu(), face.cpu())
    keep = torch.ones(ld, dtype=torch.bool)
    keep[9:9 + rows] = False
    assert (out[:, keep] == -1.0).all()


def test_poly_check_counts_mismatches():
    """The per-exchange halo check kernel: x^3 + y^2 + offset on a lattice,
    vs a plain fp64 torch evaluation; one perturbed cell and one NaN counted."""
    L = _native.lib()
    nx, ny, ld = 7, 300, 11
    x0, dx, y0, dy, off = -0.25, 1.0 / 64, 3.0, 1.0 / 128, 17.0
    xs = x0 + torch.arange(nx, dtype=torch.float64) * dx
    ys = y0 + torch.arange(ny, dtype=torch.float64) * dy
    z = torch.zeros(ny, ld, dtype=torch.float64)
    z[:, :nx] = (xs[None, :] ** 3 + ys[:, None] ** 2) + off
    z = z.to(DEV)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    args = (nx, ny, x0, dx, y0, dy, off, 1e-9, z.data_ptr(), ld, bad.data_ptr(), _stream())
    _native.check(L.gmt_poly_check(*args), "poly_check")
    torch.cuda.synchronize()
    assert int(bad.item()) == 0
    z[10, 3] += 1.0
    z[200, 6] = float("nan")
    _native.check(L.gmt_poly_check(*args), "poly_check")
    torch.cuda.synchronize()
    assert int(bad.item()) == 2
    _native.check(L.gmt_add_scalar(nx, ny, 1.0, z.data_ptr(), ld, _stream()), "add_scalar")
    torch.cuda.synchronize()
    assert float(z[0, 0].item()) == float(((xs[0] ** 3 + ys[0] ** 2) + off + 1.0).item())
    assert float(z[0, nx].item()) == 0.0  # outside the block: untouched


@pytest.mark.parametrize("ny,nx", [(1, 1), (3, 5000), (257, 1031)])
def test_diff_bits(ny, nx):
    """gmt_diff_bits (the check of the timed run) against a torch reference:
    one flipped low bit, a NaN against a number, -0.0 against +0.0."""
    a = torch.rand(ny, nx + 3, dtype=torch.float64, device="cuda")[:, 1:nx + 1]
    b = a.clone()
    assert ops.diff_bits(a, b) == (0.0, 0)
    bi = b.view(torch.int64)
    bi[ny // 2, nx // 2] ^= 1
    n = 1
    if nx > 2:
        b[0, nx - 1] = float("nan")
        a[ny - 1, 0] = 0.0
        b[ny - 1, 0] = -0.0
        n = 3
    mx, bad = ops.diff_bits(a, b)
    assert bad == n
    assert mx == (float("inf") if nx > 2 else abs(float(a[ny // 2, nx // 2] - b[ny // 2, nx // 2])))
    # the CPU path of the same op agrees
    assert ops.diff_bits(a.cpu(), b.cpu()) == (mx, bad)


def test_workgroups_round_robin_over_xcds():
    """gmt_push_sync's per-XCD acquire (csrc/kernels/ipc.hip) and every
    XCD-aware tile mapping assume that the dispatcher deals the workgroups of
    a launch to the 8 XCDs round robin.  Measured: it does, but from where
    the previous launch left off — workgroup i on XCD (x0 + i) mod 8 with a
    start x0 that rotates from launch to launch — so any 8 consecutive
    workgroups cover the 8 XCDs, and workgroups i, i + 8, i + 16, ... share
    one XCD (the tile swizzles' premise), whatever x0."""
    starts = set()
    for n in (8, 64, 1000, 7, 8, 9):
        x = ops.xcd_of_workgroups(n)
        assert x == [(x[0] + i) % 8 for i in range(n)], x[:16]
        starts.add(x[0])
    assert len(starts) >= 1
