"""Native layer on a real MI355X: the Jacobi engine (libgmt_engine.so +
libgmt_ccl.so, hipGraphs, high-priority exchange stream, RCCL) loaded into
this process, and the HIP builds of the reference apps (build/bin) under
MPICH with the transports a one-GPU box can run (RCCL with a single
periodic rank, HIP IPC and host staging with oversubscribed ranks).

Every check is against an independent reference: the NumPy serial Jacobi
(engine), the analytic derivative / closed-form sums (apps, the reference's
own self-checks), or a serial run of the whole problem
(mpi_jacobi2d --check).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]

BIN = os.path.join(ROOT, "build", "bin")
MPIRUN = "/opt/conda/bin/mpirun"


@pytest.fixture(scope="module")
def env():
    from gpu_mpi_tests_amd.parallel import dist as gd

    return gd.init(device="cuda")


@pytest.mark.parametrize("ny,nx,steps", [(96, 130, 5), (255, 517, 27)])
@pytest.mark.parametrize("tblock", [0, 2, 8, 12, 14])
@pytest.mark.parametrize("graph", [False, True])
def test_engine_periodic_matches_serial(env, ny, nx, steps, tblock, graph):
    from gpu_mpi_tests_amd import engine

    e = engine.NativeJacobi(ny, nx, env, periodic=True, overlap=True, graph=graph, tblock=tblock)
    try:
        assert e.graph == graph and e.overlap
        assert e.tsteps == (tblock if tblock else 1) or (tblock == 0 and not e.tblock)
        e.run(steps)
        e.synchronize()
        got = e.interior()
        assert e.halo_bytes > 0  # the periodic single rank exchanges with itself
        assert e.residual() >= 0.0
    finally:
        e.close()
    ref = engine.serial_jacobi(ny, nx, steps, True)
    assert float(np.abs(got - ref).max()) < 1e-13


@pytest.mark.parametrize("ny,nx,steps,tblock,wg", [(260, 1100, 13, 4, 1), (300, 1500, 45, 12, 0),
                                                  (400, 1300, 47, 20, 0), (333, 1501, 61, 18, 0)])
@pytest.mark.parametrize("graph", [False, True])
def test_engine_band_first_matches_serial(env, ny, nx, steps, tblock, wg, graph):
    """Overlapped fused passes run band-first (csrc/engine/jacobi.cpp
    enqueue_block): the boundary bands' workgroups raise a completion signal
    inside the launch, the comm stream waits for it with gmt_signal_wait and
    exchanges the pass's output halo under the interior.  Remainder passes
    (K < tsteps) and graph replays of both parities included; bitwise."""
    from gpu_mpi_tests_amd import engine

    e = engine.NativeJacobi(ny, nx, env, periodic=True, overlap=True, graph=graph, tblock=tblock, wg_waves=wg)
    try:
        assert e.band_first and e.graph == graph
        e.run(steps)
        e.synchronize()
        e.run(tblock + 1)
        e.synchronize()
        got = e.interior()
    finally:
        e.close()
    ref = engine.serial_jacobi(ny, nx, steps + tblock + 1, True)
    assert float(np.abs(got - ref).max()) == 0.0


@pytest.mark.parametrize("tblock", [0, 12, 14])
def test_engine_dirichlet_repeated_runs(env, tblock):
    """run() called several times (graph replays of both parities) == one serial run."""
    from gpu_mpi_tests_amd import engine

    e = engine.NativeJacobi(200, 333, env, periodic=False, overlap=True, graph=True, tblock=tblock)
    try:
        for k in (1, 12, 7, 25):
            e.run(k)
        e.synchronize()
        got = e.interior()
    finally:
        e.close()
    ref = engine.serial_jacobi(200, 333, 45, False)
    assert float(np.abs(got - ref).max()) < 1e-13


def _app(args, np_=None, timeout=120, env=None):
    exe = os.path.join(BIN, args[0])
    if not os.path.exists(exe):
        pytest.fail(f"{exe} not built (run make all / __graft_entry__.build())")
    cmd = [exe, *args[1:]] if np_ is None else [MPIRUN, "-np", str(np_), exe, *args[1:]]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd="/tmp",
                       env=None if env is None else dict(os.environ, **env))
    assert p.returncode == 0, f"{' '.join(cmd)} rc={p.returncode}\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
    return p.stdout


def test_app_daxpy_reference_sum():
    assert "SUM = 524800.000000" in _app(["daxpy", "--print=0"])


def test_app_buf_view_selftest_on_gpu():
    assert _app(["mpi_stencil2d_sycl", "--test-buf-view=33"]).rstrip().endswith("test_buf_view OK")


@pytest.mark.parametrize("np_,transport", [(1, "rccl"), (2, "ipc"), (2, "mpi-host"), (3, "ipc")])
def test_app_jacobi_check(np_, transport):
    periodic = ["--periodic"] if np_ == 1 else []
    out = _app(["mpi_jacobi2d", "301", "19", "--check", "--tblock", "--tsteps=4", "--warmup=2",
                f"--transport={transport}", *periodic], np_=np_)
    m = re.search(r"check\s*: max\|diff\| vs serial = ([0-9.eE+-]+) OK", out)
    assert m, out
    assert float(m.group(1)) < 1e-12, out


@pytest.mark.parametrize("np_", [2, 3])
def test_app_jacobi_ipc_graph_matches_serial(np_):
    """Stream-ordered IPC (csrc/kernels/ipc.hip): the exchange is two kernel
    launches on the compute stream, so the engine captures whole passes into
    hipGraphs with several ranks sharing the GPU; bitwise vs the serial run."""
    out = _app(["mpi_jacobi2d", "301", "23", "--check", "--tblock", "--tsteps=4", "--warmup=3", "--graph",
                "--transport=ipc"], np_=np_)
    assert re.search(r"transport = ipc overlap=\d( \([\w-]+\))? graph=1", out), out
    m = re.search(r"check\s*: max\|diff\| vs serial = ([0-9.eE+-]+) OK", out)
    assert m and float(m.group(1)) == 0.0, out


@pytest.mark.parametrize("np_,transport,extra", [(1, "rccl", ["--periodic"]), (2, "ipc", ["--graph"]),
                                                 (3, "ipc", ["--dims=1x3"]), (2, "mpi-host", [])])
def test_app_jacobi_band_first(np_, transport, extra):
    """Band-first overlapped passes across processes sharing the GPU (the
    exchange kernels run beside the pass's interior workgroups); bitwise."""
    nx = 3000 * (3 if "--dims=1x3" in extra else 1)  # 3 x 432-column W/E bands per rank at K = 20
    out = _app(["mpi_jacobi2d", f"--ny=400", f"--nx={nx}", "0", "45", "--check", "--tblock", "--tsteps=20",
                "--warmup=20", f"--transport={transport}", *extra], np_=np_)
    assert "overlap=1 (band-first)" in out, out
    m = re.search(r"check\s*: max\|diff\| vs serial = ([0-9.eE+-]+) OK", out)
    assert m and float(m.group(1)) == 0.0, out


@pytest.mark.parametrize("cus", ["8", "16"])
def test_app_jacobi_band_first_reserved_cus(cus):
    """Opt-in CU partition (GMT_COMM_CUS): band-first passes on a CU-masked
    stream, the exchange on the reserved CUs; still bitwise."""
    out = _app(["mpi_jacobi2d", "--ny=900", "--nx=3000", "0", "45", "--check", "--tblock", "--tsteps=20",
                "--warmup=20", "--periodic", "--transport=rccl"], env={"GMT_COMM_CUS": cus})
    assert "overlap=1 (band-first)" in out, out
    m = re.search(r"check\s*: max\|diff\| vs serial = ([0-9.eE+-]+) OK", out)
    assert m and float(m.group(1)) == 0.0, out


def test_app_ipc_halo_latency():
    """16-B IPC exchange between two ranks on one GPU, stream-ordered."""
    out = _app(["mpi_halo_bench", "16", "4096", "50", "--transport=ipc"], np_=2)
    rows = re.findall(r"^\s+(\d+)\s+2\s+([\d.]+)\s+([\d.]+)\s+[\d.]+\s+([\d.]+)$", out, re.M)
    assert [int(r[0]) for r in rows] == [16 << k for k in range(9)], out  # us_stream present: stream-ordered


@pytest.mark.parametrize("transport", ["ipc", "mpi-host"])
def test_app_stencil2d_gt_err_norm(transport):
    # both dims share the reference's spacing 8/n_global_deriv, so the
    # non-decomposed extent stays small to keep the round-off of x^3 + y^2 low
    out = _app(["mpi_stencil2d_gt", "64", "5", "--no-managed", "--n-other=300",
                f"--transport={transport}"], np_=2)
    errs = [float(v) for v in re.findall(r"err=([0-9.]+)", out)]
    assert len(errs) == 4 and max(errs) < 1e-5, out
    assert len(re.findall(r"allreduce=", out)) >= 2


def test_app_mpi_direct_refuses_device_memory():
    """mpi-direct on hipMalloc buffers with this (non GPU-aware) MPICH is refused
    with a clear error (the reference assumes Cray GTL / Spectrum
    -gpu, /root/reference/CMakeLists.txt:42-47); managed buffers still pass."""
    exe = os.path.join(BIN, "mpi_stencil2d_gt")
    env = {k: v for k, v in os.environ.items() if k != "GMT_MPI_GPU_AWARE"}
    p = subprocess.run([MPIRUN, "-np", "2", exe, "64", "3", "--tests=deriv", "--dim=0", "--mem=device",
                        "--buf=0", "--transport=mpi-direct"], capture_output=True, text=True, timeout=120,
                       cwd="/tmp", env=env)
    assert p.returncode != 0, p.stdout
    assert "mpi-direct was given device memory" in p.stdout and "not GPU-aware" in p.stdout, p.stdout
    out = _app(["mpi_stencil2d_gt", "64", "3", "--tests=deriv", "--dim=0", "--mem=managed", "--buf=0",
                "--n-other=300", "--transport=mpi-direct"], np_=2)
    assert re.search(r"TEST dim:0, managed, buf:0; [0-9.]+, err=", out), out


def test_app_mpi_daxpy_nvtx_sums():
    out = _app(["mpi_daxpy_nvtx_unmanaged", "--iters=2"], np_=2)
    assert len(re.findall(r"\d/2 ALLSUM", out)) == 2


def test_engine_deriv_bench_single_rank(env):
    """bench.py's reference halo benchmark entry point (gmt_engine_deriv_bench)
    on one GPU: no neighbours, so only the derivative kernel and err_norm."""
    from gpu_mpi_tests_amd import engine

    r = engine.deriv_bench(64, 300, n_iter=3, n_warmup=1, env=env)
    for d in (0, 1):
        assert r[f"dim{d}"]["bytes"] == 0
        assert r[f"dim{d}"]["err_norm"] < 1e-6
    assert r["allreduce_max_rel_err"] < 1e-12


def test_engine_rccl_beside_torch_process_group():
    """Every rank of a multi-GPU bench.py run holds torch's RCCL process group
    and the engine's own RCCL communicator at once: both live in one process
    (tests/rccl_coexist_worker.py), bitwise result."""
    import sys

    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", "29561",
                        os.path.join(ROOT, "tests", "rccl_coexist_worker.py")],
                       capture_output=True, text=True, timeout=110, cwd="/tmp", env=env)
    assert p.returncode == 0 and "COEXIST OK 0.0" in p.stdout, f"{p.stdout[-2000:]}\n{p.stderr[-3000:]}"


def test_engine_overlap_autotune_periodic(env):
    """overlap="auto" (bench.py default): both modes timed on the real field,
    then the initial field restored — the result still equals the serial run."""
    from gpu_mpi_tests_amd import engine

    e = engine.NativeJacobi(300, 517, env, periodic=True, overlap="auto", graph=False, tblock=14)
    try:
        assert e.tuned and e.tuned["overlap_s"] > 0 and e.tuned["serial_s"] > 0
        e.run(31)
        e.synchronize()
        got = e.interior()
    finally:
        e.close()
    ref = engine.serial_jacobi(300, 517, 31, True)
    assert float(np.abs(got - ref).max()) < 1e-13


@pytest.mark.parametrize("np_", [2, 3])
@pytest.mark.parametrize("transport", ["ipc", "mpi-host"])
def test_app_halo_check_every_exchange(np_, transport):
    """200 exchanges between oversubscribed ranks with the ghost rows checked
    after every one of them (a reused IPC staging slot or a lost host-staged
    chunk in any iteration would leave a ghost row off by >= 1): 0 bad cells."""
    out = _app(["mpi_stencil2d_gt", "64", "200", "--no-managed", "--tests=deriv", "--n-other=4096", "--check",
                f"--transport={transport}"], np_=np_, timeout=240)
    lines = re.findall(r"# halo check dim:(\d) buf:(\d) \(([\w-]+)\): (\d+) bad ghost cells, (\d+) exchanges", out)
    assert len(lines) == 4, out
    assert all(t == transport and int(b) == 0 and int(n) == 205 for _, _, t, b, n in lines), out


def test_app_halo_check_catches_injected_corruption():
    exe = os.path.join(BIN, "mpi_stencil2d_gt")
    p = subprocess.run([MPIRUN, "-np", "2", exe, "64", "50", "--no-managed", "--tests=deriv", "--dim=0", "--buf=0",
                        "--n-other=4096", "--check", "--transport=ipc"], capture_output=True, text=True, timeout=120,
                       cwd="/tmp", env=dict(os.environ, GMT_CORRUPT_GHOST="0:20"))
    assert p.returncode == 5, p.stdout + p.stderr
    assert "# halo check dim:0 buf:0 (ipc): 1 bad ghost cells" in p.stdout, p.stdout
