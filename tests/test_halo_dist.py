"""Distributed halo exchange + Jacobi correctness on CPU ranks (gloo), world 2..4.

The CPU analogue of the reference's de-facto distributed correctness test:
a wrong exchange shows up as O(1) errors at slab edges."""
import pytest
import torch

from mp_util import run_dist


def _halo_check(env, ny, nx, dims, gy, gx, staging):
    from gpu_mpi_tests_amd.parallel.decomp import CartDecomp
    from torch_ref.field import Field2D
    from torch_ref.halo import HaloExchanger

    d = CartDecomp.create(env.world_size, env.rank, ny, nx, dims)
    (oy, ly), (ox, lx) = d.local_y, d.local_x
    f = Field2D(ly, lx, gy, gx, fill=-1.0)
    Y = torch.arange(oy, oy + ly, dtype=torch.float64).view(-1, 1)
    X = torch.arange(ox, ox + lx, dtype=torch.float64).view(1, -1)
    f.interior.copy_(Y * 10000 + X)
    ex = HaloExchanger(d, f, staging=staging)
    for _ in range(3):  # repeated exchanges must be idempotent
        ex.exchange()
    nb = d.neighbors()
    errs = 0
    # y ghosts
    for side, rows in (("north", range(-gy, 0)), ("south", range(ly, ly + gy))):
        for r in rows:
            got = f.rows(r, 1)[0]
            if nb[side] is None:
                errs += int((got != -1.0).sum())
            else:
                errs += int((got != (oy + r) * 10000 + X[0]).sum())
    for side, cols in (("west", range(-gx, 0)), ("east", range(lx, lx + gx))):
        for c in cols:
            got = f.cols(c, 1)[:, 0]
            if nb[side] is None:
                errs += int((got != -1.0).sum())
            else:
                errs += int((got != Y[:, 0] * 10000 + (ox + c)).sum())
    return errs


@pytest.mark.parametrize("world,dims", [(2, (2, 1)), (2, (1, 2)), (3, (3, 1)), (4, (2, 2)), (4, (1, 4))])
@pytest.mark.parametrize("gy,gx", [(1, 1), (2, 2), (2, 0), (0, 2)])
def test_halo_exchange_gloo(world, dims, gy, gx, port):
    errs = run_dist(_halo_check, world, port, 37, 53, dims, gy, gx, "none")
    assert errs == [0] * world


@pytest.mark.parametrize("staging", ["device"])
def test_halo_exchange_staged(staging, port):
    errs = run_dist(_halo_check, 4, port, 40, 44, (2, 2), 2, 2, staging)
    assert errs == [0] * 4


def _jacobi_run(env, n, dims, overlap, steps, rhs):
    from torch_ref.jacobi import Jacobi2D

    s = Jacobi2D(n, n + 6, env=env, dims=dims, overlap=overlap, rhs=rhs)
    s.run(steps)
    g = s.gather_global()
    res = s.global_residual()
    return (g, res)




@pytest.mark.parametrize("world,dims", [(2, None), (4, (2, 2)), (4, (4, 1)), (3, (1, 3))])
@pytest.mark.parametrize("overlap", [True, False])
def test_jacobi_distributed_equals_serial(world, dims, overlap, port):
    n, steps = 24, 9
    outs = run_dist(_jacobi_run, world, port, n, dims, overlap, steps, False)
    g_dist, res_dist = outs[0]
    # serial reference with the same initial data: assemble the per-rank seeded init globally
    from gpu_mpi_tests_amd.parallel.decomp import CartDecomp
    from torch_ref.field import Field2D
    from gpu_mpi_tests_amd.ops import reference as ref

    nx = n + 6
    u = Field2D(n, nx, 1, 1)
    for r in range(world):
        d = CartDecomp.create(world, r, n, nx, dims)
        (oy, ly), (ox, lx) = d.local_y, d.local_x
        gen = torch.Generator().manual_seed(1234 + r)
        u.interior[oy:oy + ly, ox:ox + lx] = torch.rand(ly, lx, generator=gen, dtype=torch.float64)
    u.rows(-1, 1).fill_(1.0)
    un = Field2D(n, nx, 1, 1)
    un.storage.copy_(u.storage)
    for _ in range(steps):
        ref.jacobi5(u.storage, un.storage, *u.region())
        u, un = un, u
    assert torch.equal(g_dist, u.interior), (g_dist - u.interior).abs().max()
    r = ref.jacobi5(u.storage, un.storage, *u.region())
    assert abs(res_dist - float(r.sqrt())) < 1e-12 * max(1.0, float(r.sqrt()))
