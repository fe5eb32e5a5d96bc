"""Golden-output and distributed-correctness tests of the native apps.

The apps run on the CPU backend (build/bin-host: the same sources linked
against the host runtime, the analogue of the reference's gtensor `host`
build, /root/reference/CMakeLists.txt:59-69) under MPICH with 1-4 ranks.
Report-line formats follow the reference binaries; the
values are the reference's closed forms: DAXPY sums, the
analytic derivative of x^3 + y^2 (err_norm at round-off), and for the Jacobi
engine a bit-level comparison with a serial run of the whole problem.
"""
import re

import pytest

from native_util import have_mpi, run_app

pytestmark = pytest.mark.skipif(not have_mpi(), reason="mpirun not available")


def test_daxpy_reference_sum():
    out = run_app("daxpy").stdout.splitlines()
    assert len(out) == 1025
    assert out[0] == "1.000000" and out[1023] == "1024.000000"
    assert out[-1] == "SUM = 524800.000000"  # daxpy.cu:87, n(n+1)/2


def test_daxpy_large_host_path_and_rate():
    # BASELINE config "daxpy N=1M fp64 on CPU host path (plumbing)"
    out = run_app("daxpy", "--n=1048576", "--iters=3").stdout
    assert "SUM = 549756338176.000000" in out
    assert re.search(r"# DAXPY n=1048576 impl=gmt backend=host: median [\d.]+ ms", out)


def test_daxpy_nvtx_same_output():
    out = run_app("daxpy_nvtx").stdout.splitlines()
    assert out[-1] == "SUM = 524800.000000"


def test_mpi_daxpy_managed_probe():
    out = run_app("mpi_daxpy", np=2).stdout
    assert "MEMORY_PER_CORE is not set" in out
    assert re.search(r"RANK\[1/2\] => DEVICE\[1/1\] mem=\d+", out)
    assert re.search(r"RANK\[2/2\] => DEVICE\[1/1\] mem=\d+", out)
    for r in range(2):
        assert f"{r}/2 SUM = 524800.000000" in out
    assert "HIP PreferredLocation of 'm_x' is CPU (-1)" in out
    assert "HIP PreferredLocation of 'd_x' is UNMANAGED" in out
    assert "HIP PreferredLocation of 'x' is NOT HIP" in out


def test_mpi_daxpy_memory_per_core_env():
    out = run_app("mpi_daxpy", np=1, env={"MEMORY_PER_CORE": "4096"}).stdout
    assert "MEMORY_PER_CORE=4096" in out


@pytest.mark.parametrize("np_,transport", [(1, "auto"), (3, "auto"), (3, "rccl")])
def test_mpi_daxpy_bench_allreduce(np_, transport, tmp_path):
    """BASELINE config "mpi_daxpy N ranks x 1 GPU, allreduce of partial sums":
    timed DAXPY + device partial sum + transport all-reduce, ALLSUM checked."""
    j = tmp_path / "d.jsonl"
    out = run_app("mpi_daxpy", "--bench=50000", "--iters=4", f"--json={j}", f"--transport={transport}",
                  np=np_).stdout
    assert re.search(r"BENCH daxpy n=50000 per rank x %d ranks: [\d.]+ ms/call" % np_, out)
    m = re.search(r"ALLSUM = (\S+) \(expected (\S+), rel err \S+\) OK", out)
    assert m and abs(float(m.group(1)) - 9 * 50001 / 2 * np_) < 1e-6 * np_ * 50001 * 9
    import json
    rec = json.loads(j.read_text().splitlines()[0])
    assert rec["ranks"] == np_ and rec["GBps_aggregate"] > 0


def test_mpi_stencil2d_alias():
    out = run_app("mpi_stencil2d", "40", "4", "--check", np=2).stdout
    assert "OK" in out and "MLUPS" in out


def test_mpi_daxpy_gt_every_rank():
    out = run_app("mpi_daxpy_gt", np=3).stdout
    for r in range(3):
        assert f"{r}/3 [0:0x00000000] SUM = 524800.000000" in out


@pytest.mark.parametrize("variant", ["mpi_daxpy_nvtx_managed", "mpi_daxpy_nvtx_unmanaged"])
@pytest.mark.parametrize("np_,transport", [(1, "auto"), (2, "auto"), (3, "auto"), (3, "rccl")])
def test_mpi_daxpy_nvtx_sums_and_times(variant, np_, transport):
    per_node = 1200
    out = run_app(variant, f"--n-per-node={per_node}", "--iters=2", f"--transport={transport}",
                  np=np_).stdout
    n = per_node // np_
    assert f"1 nodes, {np_} ranks, {n} elements each, total {per_node}" in out
    for r in range(np_):
        assert f"{r}/{np_} SUM = {(n + 1) / 2:f}" in out          # mpi_daxpy_nvtx.cc:268
        assert f"{r}/{np_} ALLSUM = {np_ * (n + 1) / 2:f}" in out  # :310
        for what in ("total  ", "kernel ", "barrier", "gather "):
            assert re.search(rf"{r}/{np_} TIME {what}: \d+\.\d{{3}}", out), what


def test_mpienv_fortran_layout():
    out = run_app("mpienv", np=2, env={"MEMORY_PER_CORE": "2048"}).stdout
    assert " rank            0  MEMORY_PER_CORE=        2048" in out
    assert " rank            1  MEMORY_PER_CORE=        2048" in out
    # Fortran (i6) read of a 5-char buffer: blank -> 0, longer values truncated
    out = run_app("mpienv", np=1, env={"MEMORY_PER_CORE": ""}).stdout
    assert "MEMORY_PER_CORE=           0" in out
    out = run_app("mpienv", np=1, env={"MEMORY_PER_CORE": "1234567"}).stdout
    assert "MEMORY_PER_CORE=       12345" in out


@pytest.mark.parametrize("np_", [1, 2, 3])
def test_mpigatherinplace_integer_division(np_):
    n = 1000
    out = run_app("mpigatherinplace", f"--n={n}", np=np_).stdout
    # allx(rank*N+i) = rank*i/N, integer division, i = 1..N (mpigatherinplace.f90:35)
    lsums = [sum((r * i) // n for i in range(1, n + 1)) for r in range(np_)]
    for r in range(np_):
        m = re.search(rf"^\s+{r} /\s+{np_}\s+(\S+)\s+(\S+)$", out, re.M)
        assert m, out
        assert float(m.group(1)) == lsums[r]
        assert float(m.group(2)) == sum(lsums)


@pytest.mark.parametrize("np_", [1, 2, 4])
def test_mpi_stencil_gt_1d(np_):
    out = run_app("mpi_stencil_gt", "1", "--iters=5", np=np_).stdout
    assert f"n procs  = {np_}" in out and "n_global = 1048576" in out
    assert f"n_local  = {1048576 // np_}" in out
    errs = [float(v) for v in re.findall(r"err_norm = ([\d.]+)", out)]
    assert len(errs) == np_ and max(errs) < 1e-4  # exact for x^3 up to round-off
    assert len(re.findall(rf"\d/{np_} exchange time \d+\.\d{{8}}", out)) == np_
    if np_ > 1:
        assert "16-byte halo exchange transport=mpi-direct" in out


def test_mpi_stencil_gt_divisibility_error():
    p = run_app("mpi_stencil_gt", "--n=1000", np=3, check=False)
    assert p.returncode != 0
    assert "must be divisor of domain size" in p.stdout


# the reference's fields, then optional bracketed tags where the timing
# semantics differ from the reference's (csrc/apps/mpi_stencil2d_gt.cpp header)
_TAGS = r"((?: \[[^\]]+\])*)"
_TEST_RE = re.compile(r"^TEST dim:(\d), (device |managed), buf:(\d); ([\d.]+), err=([\d.]+)" + _TAGS + "$", re.M)
_SUM_RE = re.compile(r"^TEST dim:(\d), (device |managed), buf:0; allreduce=([\d.]+)" + _TAGS + "$", re.M)


@pytest.mark.parametrize("np_", [1, 2, 3])
def test_mpi_stencil2d_gt_all_variants(np_):
    out = run_app("mpi_stencil2d_gt", "48", "6", "--n-other=300", np=np_).stdout
    assert f"n procs        = {np_}" in out
    assert f"n_global_deriv = {48 * np_}" in out and "n_global_other = 300" in out
    tests = _TEST_RE.findall(out)
    # 8 test_deriv lines in the reference order (mpi_stencil2d_gt.cc:692-716)
    assert [(d, m, b) for d, m, b, _, _, _ in tests] == [
        ("0", "device ", "1"), ("0", "device ", "0"), ("0", "managed", "1"), ("0", "managed", "0"),
        ("1", "device ", "1"), ("1", "device ", "0"), ("1", "managed", "1"), ("1", "managed", "0")]
    for *_, err, tags in tests:
        assert float(err) < 1e-5
        assert tags == " [persistent buffers]"  # host backend: managed memory is plain host memory
    sums = _SUM_RE.findall(out)
    assert [(d, m) for d, m, _, _ in sums] == [("0", "device "), ("0", "managed"),
                                               ("1", "device "), ("1", "managed")]
    assert "WARNING" not in out  # all-reduce values checked against PI*n_other


@pytest.mark.parametrize("transport", ["mpi-host", "mpi-direct", "ipc", "rccl"])
def test_mpi_stencil2d_gt_transport_parity(transport):
    out = run_app("mpi_stencil2d_gt", "40", "4", "--n-other=256", "--no-managed",
                  f"--transport={transport}", "--host-init", "--host-verify", np=3).stdout
    tests = _TEST_RE.findall(out)
    assert len(tests) == 4
    for *_, err, _tags in tests:
        assert float(err) < 1e-5


def test_mpi_stencil2d_gt_matrix_slice():
    """--dim/--mem/--buf select one cell of the reference's test matrix."""
    out = run_app("mpi_stencil2d_gt", "32", "--iters=3", "--warmup=1", "--n-other=128", "--dim=1",
                  "--mem=managed", "--buf=0", np=2).stdout
    tests = _TEST_RE.findall(out)
    assert [(d, m, b) for d, m, b, _, _, _ in tests] == [("1", "managed", "0")]
    assert [(d, m) for d, m, _, _ in _SUM_RE.findall(out)] == [("1", "managed")]
    assert "n_iter         = 3" in out and "n_warmup       = 1" in out


def test_mpi_stencil2d_gt_alloc_per_call_is_untagged():
    """--alloc-per-call times the reference's per-call buffer creation: the TEST
    lines then carry exactly the reference's fields."""
    out = run_app("mpi_stencil2d_gt", "32", "3", "--n-other=128", "--no-managed", "--alloc-per-call",
                  "--transport=mpi-host", np=2).stdout
    # the header carries the reference's n_warmup byte for byte (mpi_stencil2d_gt.cc:658,687)
    assert "n_warmup       = 10\n" in out
    tests = _TEST_RE.findall(out)
    assert len(tests) == 4 and all(t[-1] == "" for t in tests)


def test_mpi_stencil2d_gt_json(tmp_path):
    j = tmp_path / "r.jsonl"
    run_app("mpi_stencil2d_gt", "32", "3", "--n-other=128", "--no-managed", f"--json={j}", np=2)
    import json
    recs = [json.loads(line) for line in j.read_text().splitlines()]
    assert len(recs) == 6
    assert {r["test"] for r in recs} == {"deriv", "sum"}
    assert all(r["ranks"] == 2 for r in recs)


@pytest.mark.parametrize("stage", ["0", "1"])
def test_mpi_stencil2d_sycl(stage):
    out = run_app("mpi_stencil2d_sycl", "32", stage, "5", "--ny=200", np=2).stdout
    assert "nx_global  = 64" in out and f"stage_host = {stage}" in out
    assert re.search(r"dev bytes  = [\d.]+ MB", out)
    assert len(re.findall(r"\d/2 exchange time \d+\.\d{8} ms", out)) == 2
    errs = [float(v) for v in re.findall(r"err_norm = ([\d.]+)", out)]
    assert len(errs) == 2 and max(errs) < 1e-6


@pytest.mark.parametrize("n", [None, "9"])
def test_mpi_stencil2d_sycl_buf_view_selftest(n):
    """Reference test_buf_view (mpi_stencil2d_sycl.cc:118-159): pack rows
    [0,2) of an n x n field, unpack a buffer into rows [n-2,n)."""
    flag = "--test-buf-view" if n is None else f"--test-buf-view={n}"
    out = run_app("mpi_stencil2d_sycl", flag).stdout
    k = 6 if n is None else int(n)
    assert out.rstrip().endswith("test_buf_view OK")
    assert len(re.findall(r"^data\[", out, re.M)) == 2 * k * k
    assert len(re.findall(r"^buf2\[", out, re.M)) == 2 * k
    assert "buf[1, 0] = -1.000000" in out
    assert f"data[{k - 1}, {k - 1}] = {100 + k - 1 + 0.1:f}" in out


def test_mpi_stencil2d_sycl_oo_strong_scaling_and_debug():
    out = run_app("mpi_stencil2d_sycl_oo", "1", "0", "5", np=2).stdout
    assert "n_global   = 1024" in out and "n_local    = 512" in out
    assert len(re.findall(r"^\d: exchange time \d+\.\d{8} ms$", out, re.M)) == 2
    # DEBUG build: domain/1024, one iteration, rank-serialised halo dumps
    out = run_app("mpi_stencil2d_sycl_oo", "8", "0", "5", "--debug", np=2).stdout
    assert "n_global   = 8" in out and "n_iter     = 1" in out
    ghost = dict(re.findall(r"^(\d: ghost \[\d, :\]) (.*)$", out, re.M))
    send = dict(re.findall(r"^(\d: send \[\d, :\]) (.*)$", out, re.M))
    # rank 0's upper ghost rows = rank 1's first interior rows and vice versa
    assert ghost["0: ghost [6, :]"] == send["1: send [2, :]"]
    assert ghost["1: ghost [1, :]"] == send["0: send [5, :]"]


@pytest.mark.parametrize("args,np_", [
    (["64", "10"], 1),
    (["64", "10", "--periodic"], 1),
    (["50", "9"], 2),
    (["50", "9", "--transport=ipc"], 2),
    (["50", "9", "--transport=mpi-host", "--no-overlap"], 2),
    (["41", "7", "--dims=2x2", "--transport=ipc"], 4),
    (["41", "7", "--dims=2x2", "--periodic"], 4),
    (["41", "7", "--dims=1x3", "--transport=mpi-host"], 3),
    (["21", "5", "--weak", "--periodic", "--transport=ipc"], 3),
    # temporal blocking: 2 sweeps per pass, 2-wide halos, corners (two-phase exchange)
    (["64", "10", "--tblock"], 1),
    (["37", "9", "--tblock", "--periodic"], 1),
    (["50", "10", "--tblock", "--transport=ipc"], 2),
    (["51", "9", "--tblock", "--periodic", "--transport=mpi-host"], 2),
    (["60", "10", "--tblock", "--dims=2x2"], 4),
    (["61", "11", "--tblock", "--dims=2x2", "--periodic", "--transport=ipc"], 4),
    (["45", "8", "--tblock=8", "--dims=2x3", "--periodic"], 6),
    (["45", "8", "--tblock=32", "--dims=1x3", "--no-overlap"], 3),
    # 3 and 4 sweeps per pass (ghost width 3/4, odd K stages an even-aligned ring)
    (["64", "13", "--tblock", "--tsteps=3"], 1),
    (["64", "13", "--tblock", "--tsteps=4", "--periodic"], 1),
    (["61", "11", "--tblock", "--tsteps=3", "--dims=2x2", "--periodic", "--transport=ipc"], 4),
    (["70", "10", "--tblock", "--tsteps=4", "--dims=2x3"], 6),
    (["50", "10", "--tblock", "--tsteps=4", "--transport=mpi-host"], 3),
    # 6 and 8 sweeps per pass (register-pipelined kernel on the GPU); 13 steps
    # = one 8-pass + a 4-sweep remainder pass + one single sweep
    (["64", "13", "--tblock", "--tsteps=8"], 1),
    (["70", "13", "--tblock", "--tsteps=6", "--periodic"], 1),
    (["75", "17", "--tblock", "--tsteps=8", "--dims=2x2", "--periodic", "--transport=ipc"], 4),
    (["80", "12", "--tblock", "--tsteps=6", "--dims=1x2"], 2),
    # rccl transport (host backend: the RCCL semantics over Unix sockets,
    # csrc/host/ccl_host.cpp) — the data plane of the multi-GPU runs
    (["50", "10", "--tblock", "--transport=rccl"], 2),
    (["41", "7", "--dims=2x2", "--transport=rccl"], 4),
    (["41", "7", "--dims=1x2", "--periodic", "--transport=rccl"], 2),
    (["61", "11", "--tblock", "--tsteps=12", "--dims=2x2", "--periodic", "--transport=rccl"], 4),
    (["45", "8", "--tblock=8", "--dims=2x3", "--periodic", "--transport=rccl"], 6),
    # 10 and 12 sweeps per pass: 10/12-wide halos and corners
    (["90", "25", "--tblock", "--tsteps=12"], 1),
    (["96", "23", "--tblock", "--tsteps=10", "--dims=2x2", "--periodic", "--transport=ipc"], 4),
    (["100", "26", "--tblock", "--tsteps=12", "--dims=1x2"], 2),
    # band-first overlapped passes (ranks wide enough for boundary bands and
    # an interior): the pass's output halo is exchanged under its interior
    (["--ny=200", "--nx=1600", "0", "13", "--tblock", "--tsteps=4", "--wg-strips=1", "--dims=2x2", "--periodic",
      "--transport=ipc"], 4),
    (["--ny=240", "--nx=1500", "0", "27", "--tblock", "--tsteps=12", "--wg-strips=1", "--dims=2x2"], 4),
    (["--ny=150", "--nx=2400", "0", "15", "--tblock", "--tsteps=6", "--wg-strips=1", "--dims=1x3",
      "--transport=rccl"], 3),
    (["--ny=400", "--nx=300", "0", "17", "--tblock", "--tsteps=8", "--wg-strips=1", "--dims=2x1",
      "--transport=mpi-host"], 2),
    (["--ny=130", "--nx=800", "0", "11", "--tblock", "--tsteps=5", "--wg-strips=1", "--periodic"], 1),
    # one periodic axis: y-only gives S/N-only shares (row bands, no W/E
    # bands); x-only needs the x faces to carry the corner rows when the rank
    # has no y neighbours (Halo2D x_full)
    (["--ny=300", "--nx=700", "0", "13", "--tblock", "--tsteps=6", "--wg-strips=1", "--dims=2x1",
      "--periodic=y", "--transport=ipc"], 2),
    (["--ny=260", "--nx=900", "0", "9", "--tblock", "--tsteps=4", "--wg-strips=1", "--periodic=y"], 1),
    (["--ny=200", "--nx=1600", "0", "11", "--tblock", "--tsteps=5", "--wg-strips=1", "--dims=1x2",
      "--periodic=x", "--transport=ipc"], 2),
    (["53", "9", "--tblock", "--dims=2x2", "--periodic=x"], 4),
    (["47", "7", "--dims=1x3", "--periodic=y", "--transport=mpi-host"], 3),
])
def test_mpi_jacobi2d_matches_serial(args, np_):
    out = run_app("mpi_jacobi2d", *args, "--check", "--warmup=2", "--halo-iters=3", np=np_).stdout
    m = re.search(r"check     : max\|diff\| vs serial = (\S+) OK", out)
    assert m, out
    if args[0].startswith("--ny="):  # sized for the band-first pass
        assert "overlap=1 (band-first)" in out, out
    assert re.search(r"MLUPS     : [\d.]+", out)


@pytest.mark.parametrize("transport,np_", [("ipc", 2), ("mpi-host", 2), ("mpi-direct", 3), ("local", 1),
                                           ("rccl", 3)])
def test_mpi_halo_bench_data(transport, np_):
    out = run_app("mpi_halo_bench", "8", "65536", "3", f"--transport={transport}", np=np_).stdout
    rows = re.findall(r"^\s+(\d+)\s+2\s+[\d.]+\s+[\d.]+\s+[\d.]+\s+(?:[\d.]+|-)$", out, re.M)
    assert [int(r) for r in rows] == [8 << k for k in range(14)]
    assert "MISMATCH" not in out


def test_transport_errors_are_loud():
    # a single-process transport in a 2-rank job
    p = run_app("mpi_jacobi2d", "32", "2", "--transport=local", np=2, check=False)
    assert p.returncode != 0 and "!= world size" in p.stdout
    p = run_app("mpi_jacobi2d", "32", "2", "--transport=bogus", np=1, check=False)
    assert p.returncode != 0 and "unknown transport" in p.stdout


def test_kernel_bench_host():
    """One production kernel per entry point (the A/B variants moved to the
    GPU-only csrc/bench/variant_bench.hip); the K-sweep section runs every
    built sweep count."""
    out = run_app("gmt_kernel_bench", "--daxpy-n=4096", "--jacobi-n=64", "--iters=2",
                  "--only=daxpy,jacobi,tb", "--tb-k=1,7,12,20").stdout
    assert len(re.findall(r"^daxpy\s+v0", out, re.M)) == 1
    assert len(re.findall(r"^rocblas\s+v0", out, re.M)) == 1
    assert len(re.findall(r"^jacobi5\s+v0", out, re.M)) == 1
    assert [int(k) for k in re.findall(r"^jacobi5tb\s+v(\d+)", out, re.M)] == [1, 7, 12, 20]


def test_watchdog_aborts_hung_exchange():
    """Fault injection: rank 1 stops in its 3rd halo exchange; the --timeout
    watchdog (gmt/watchdog.hpp) names the stalled phase and MPI_Abort takes
    the whole job down instead of leaving rank 0 blocked forever."""
    p = run_app("mpi_jacobi2d", "50", "40", "--transport=ipc", "--timeout=2", np=2,
                env={"GMT_INJECT_HANG": "1:2"}, check=False, timeout=90)
    out = p.stdout + p.stderr
    assert p.returncode != 0, out
    assert "GMT FAULT INJECTION: rank 1" in out
    assert "GMT WATCHDOG: rank" in out and "no progress" in out


def test_watchdog_quiet_on_healthy_run():
    p = run_app("mpi_jacobi2d", "50", "20", "--transport=ipc", "--timeout=30", np=2)
    assert "WATCHDOG" not in p.stdout + p.stderr


@pytest.mark.parametrize("np_", [2, 3])
def test_stencil2d_gt_per_exchange_halo_check(np_):
    """--check: the ghost rows are compared with the analytic field after
    EVERY exchange (the field is raised by 1 before each one, so a ghost row
    left from an earlier exchange is wrong by 1); every test of the matrix
    reports 0 bad cells over all its exchanges."""
    out = run_app("mpi_stencil2d_gt", "16", "30", "--no-managed", "--tests=deriv", "--n-other=300", "--check",
                  np=np_).stdout
    lines = re.findall(r"# halo check dim:(\d) buf:(\d) \(([\w-]+)\): (\d+) bad ghost cells, (\d+) exchanges", out)
    assert len(lines) == 4, out
    assert all(int(b) == 0 and int(n) == 35 for _, _, _, b, n in lines), out


def test_stencil2d_gt_halo_check_catches_a_corrupt_cell():
    """Fault injection: rank 1 overwrites one ghost cell after its 7th
    exchange; the check counts it and the app exits with status 5."""
    p = run_app("mpi_stencil2d_gt", "16", "30", "--no-managed", "--tests=deriv", "--n-other=300", "--check",
                "--dim=1", np=3, env={"GMT_CORRUPT_GHOST": "1:7"}, check=False)
    assert p.returncode == 5, p.stdout + p.stderr
    assert re.findall(r"# halo check dim:1 buf:\d \([\w-]+\): 1 bad ghost cells", p.stdout), p.stdout


def test_stencil2d_sycl_halo_check():
    out = run_app("mpi_stencil2d_sycl", "64", "1", "40", "--check", np=2).stdout
    assert re.search(r"# halo check dim:0 buf:1 \(mpi-host\): 0 bad ghost cells, 45 exchanges", out), out


def test_mpi_stencil2d_gt_debug_lines():
    """--debug: the reference DEBUG build's per-rank lines (missing
    #2): "%d/%d exchange time %0.8f ms" and "%d/%d [%d:0x%08x] err_norm = %.8f"
    after every test_deriv, "%d/%d allreduce time %0.8f ms" after every
    test_sum (mpi_stencil2d_gt.cc:536-539,557-560,635-638)."""
    import re
    out = run_app("mpi_stencil2d_gt", "32", "3", "--n-other=128", "--no-managed", "--debug", np=2).stdout
    exch = re.findall(r"^(\d+)/2 exchange time (\d+\.\d{8}) ms$", out, re.M)
    errs = re.findall(r"^(\d+)/2 \[(\d+):0x([0-9a-f]{8})\] err_norm = (\d+\.\d{8})$", out, re.M)
    alls = re.findall(r"^(\d+)/2 allreduce time (\d+\.\d{8}) ms$", out, re.M)
    # 4 test_deriv (2 dims x buf 1/0) and 2 test_sum, each line once per rank
    assert sorted(r for r, _ in exch) == ["0"] * 4 + ["1"] * 4, out
    assert sorted(e[0] for e in errs) == ["0"] * 4 + ["1"] * 4 and all(float(e[3]) < 1e-5 for e in errs)
    assert sorted(r for r, _ in alls) == ["0"] * 2 + ["1"] * 2
    assert len(_TEST_RE.findall(out)) == 4 and len(_SUM_RE.findall(out)) == 2
    # without --debug: no per-rank lines
    plain = run_app("mpi_stencil2d_gt", "32", "3", "--n-other=128", "--no-managed", np=2).stdout
    assert "exchange time" not in plain and "err_norm" not in plain
