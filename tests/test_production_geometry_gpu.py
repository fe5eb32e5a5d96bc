"""The engine at the production launch geometry, on the GPU (VERDICT r05,
weak #6 / next round #1): the fused K = 20 passes over the BASELINE domains
— multi-round launches with the edges-last dispatch (``tail_swizzle``,
csrc/kernels/jacobi5tb.hpp) at 32768², the N = 8 share shapes, the 8192²
single-GPU config — against the same sweeps replayed as single sweeps
(csrc/kernels/jacobi5.hip), compared bitwise on the device
(``NativeJacobi.compare``, gmt_diff_bits).  The kernel tests
(test_jacobi_tb_gpu.py) stop at one-round domains of a few hundred rows.

Memory: two engines of a 32768² field are 4 x 8.6 GB, well inside 288 GB.
"""
import pytest
import torch

from gpu_mpi_tests_amd.engine import NativeJacobi
from gpu_mpi_tests_amd.parallel import dist as gdist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return gdist.init(device="cuda")


@pytest.mark.parametrize("ny,nx,steps,periodic,push", [
    (32768, 32768, 45, False, False),   # the driver's headline domain: 2 full passes + a remainder
    (8192, 16384, 40, False, False),    # N = 8 share, 4x2 grid
    (16384, 8192, 40, False, False),    # N = 8 share, 2x4 grid (BASELINE's)
    (8192, 8192, 60, False, False),     # BASELINE single-GPU config
    (8192, 16384, 40, True, True),      # inline halo, one rank periodic (pushes into its own buffers)
])
def test_production_geometry_bitwise(env, ny, nx, steps, periodic, push):
    eng = NativeJacobi(ny, nx, env, periodic=periodic, overlap=False, graph=False, tblock=20, init="random",
                       seed=7, calibrate=True, push=push)
    ref = None
    try:
        if push:
            assert eng.push_active
        eng.prepare(steps)
        plan = eng.plan(steps)
        assert sum(plan) == steps and max(plan) >= 16, plan  # fused passes of the production kernels
        eng.run(steps)
        eng.synchronize()
        ref = NativeJacobi(ny, nx, env, periodic=periodic, overlap=False, graph=False, tblock=False,
                           init="random", seed=7)
        ref.run(steps)
        ref.synchronize()
        mx, bad = eng.compare(ref)
        assert bad == 0 and mx == 0.0, (bad, mx, plan)
    finally:
        eng.close()
        if ref is not None:
            ref.close()
        torch.cuda.empty_cache()


def test_compare_sees_one_flipped_bit(env):
    """The comparison itself: one ulp in one interior cell is one mismatch."""
    a = NativeJacobi(512, 768, env, overlap=False, graph=False, tblock=20, init="random", seed=3)
    b = NativeJacobi(512, 768, env, overlap=False, graph=False, tblock=False, init="random", seed=3)
    try:
        assert a.compare(b) == (0.0, 0)
        a.run(1)
        b.run(1)
        a.synchronize()
        b.synchronize()
        assert a.compare(b) == (0.0, 0)
        a.run(20)
        a.synchronize()
        mx, bad = a.compare(b)
        assert bad > 0 and mx > 0
    finally:
        a.close()
        b.close()
