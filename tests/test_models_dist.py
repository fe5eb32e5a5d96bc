"""Python (torch.distributed) parity models on CPU ranks (gloo):
distributed derivative test (reference test_deriv/test_sum) and distributed
DAXPY + all-gather (reference mpi_daxpy_nvtx).  Values are the reference's
closed forms."""
import pytest

from conftest import free_port

from mp_util import run_dist


def _port():
    return free_port()


def _deriv(env, dim, n_local, n_other):
    from torch_ref import deriv

    r = deriv.run_deriv(dim, n_local, n_other, n_iter=3, n_warmup=1, env=env)
    t, err = deriv.run_sum(dim, n_local, n_other, n_iter=3, n_warmup=1, env=env)
    return r.err_norm, r.bytes_per_exchange, len(r.times), err


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("dim", [0, 1])
def test_deriv_distributed_exact(world, dim):
    out = run_dist(_deriv, world, _port(), dim, 24, 40)
    for err, nbytes, ntimes, sum_err in out:
        assert err < 1e-6          # the 4th-order stencil is exact for x^3 + y^2
        assert ntimes == 3
        assert sum_err < 1e-12     # all-reduced axis sums == PI * n_other
    if world > 1:
        assert out[0][1] == 2 * 40 * 8          # one face: 2 ghost layers x 40 x fp64
        assert out[1][1] == (2 if world > 2 else 1) * 2 * 40 * 8


def _daxpy(env, n_per_node):
    from torch_ref import daxpy_dist

    r = daxpy_dist.run(n_per_node, env=env)
    return r.n, r.sum, r.allsum, r.lines(env.rank, env.world_size)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_daxpy_dist_closed_forms(world):
    out = run_dist(_daxpy, world, _port(), 1200)
    for rank, (n, s, alls, lines) in enumerate(out):
        assert n == 1200 // world
        assert s == pytest.approx((n + 1) / 2, rel=1e-12)          # mpi_daxpy_nvtx.cc:268
        assert alls == pytest.approx(world * (n + 1) / 2, rel=1e-12)  # :310
        assert lines[0] == f"{rank}/{world} SUM = {s:f}"
        assert lines[-1].startswith(f"{rank}/{world} TIME gather : ")
