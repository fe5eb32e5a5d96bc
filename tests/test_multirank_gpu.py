"""bench.py's multi-rank flagship path on the real GPU, by oversubscription.

The 1-GPU box cannot run one rank per GPU at N > 1, and RCCL refuses two
ranks on one device.  The reference runs several ranks per GPU the same way
(mpi_daxpy.cc:43-54: ``device = rank / (n_ranks / n_devices)``), so here N
torchrun ranks share cuda:0 and the native engine's transport resolves to
HIP IPC (csrc/comm/transport_ipc.cpp; handles traded over the socket control
plane, one stream-ordered exchange kernel per halo exchange).  Every piece of
bench.py's N > 1 logic runs on the hardware: the bitwise correctness gate
(``check_max_diff``) with the job's process grid, band-first overlap, the
cross-rank overlap autotune, the blocking halo latency, the reference's own
halo benchmark (``ref_halo_*``), and the DAXPY partial-sum all-reduce checked
against the closed form (mpi_daxpy_nvtx.cc:305-310).

Each case is one torchrun job (a handful of processes on the card, well
under the box's limit), bounded by a timeout of its own.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import free_port, gpu_available

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "r03_multirank")


def _torchrun(n, args, timeout, **env):
    port = str(free_port())
    cmd = ["timeout", "-k", "10", str(timeout), sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port", port,
           os.path.join(ROOT, "bench.py"), "--gpus", str(n), *args]
    e = dict(os.environ, OMP_NUM_THREADS="1", **env)
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout + 30, cwd=ROOT, env=e)


def _record(name, rec):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"{name}.json"), "w") as f:
        f.write(json.dumps(rec) + "\n")


@pytest.fixture(autouse=True)
def _need_gpu():
    if not gpu_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("n,extra,name", [
    (2, ["--overlap", "on"], "n2_overlap_on"),
    (4, ["--dims", "2x2"], "n4_dims2x2"),
    # the driver's N = 8 launch: default 4x2 grid, BASELINE's 2x4 timed too
    (8, [], "n8_driver_shape"),
    # the inline halo through bench.py itself
    (2, ["--transport", "push", "--small-size", "0"], "n2_push"),
])
def test_bench_oversubscribed_ipc(n, extra, name):
    p = _torchrun(n, ["--size", "8192", "--steps", "20", "--warmup", "5", "--daxpy-n", str(1 << 24),
                      "--ref-iters", "20", *extra], timeout=420)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-6000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    _record(name, rec)
    assert rec["n_gpus"] == n
    push = "push" in extra
    assert rec["config"]["transport"] == ("ipc inline halo" if push else "ipc"), rec["config"]
    # the timed run itself, replayed through single sweeps + plain IPC exchanges
    assert rec["timed_check_mismatches"] == 0 and rec["timed_check_max_diff"] == 0.0, rec
    assert rec["ranks_per_gpu"] == n
    assert rec["check_max_diff"] == 0.0
    # err_norm of the reference's own benchmark at its default per-rank shape
    # (1024 x 512Ki, x^3 + y^2 at spacing 8/n_global: |z| reaches ~4e6 in dim
    # 0 and ~9e9 in dim 1): the 4th-order stencil is exact for cubics, so it
    # is round-off summed over 5e8 points (measured 4.9e-4 / 0.77), tiny
    # against the analytic derivative's norm; one missing ghost cell alone
    # would add ~|z| / (12 h) >= 1e8 (mpi_stencil2d_gt.cc:555-570)
    assert rec["ref_halo_dim0_rel_err"] < 1e-4 and rec["ref_halo_dim1_rel_err"] < 1e-4, rec
    assert rec["ref_halo_config"].endswith("ipc")
    assert rec["daxpy_allsum_rel_err"] <= 1e-9 and rec["daxpy_allreduce_kind"] == "ipc"
    assert rec["value"] > 0 and rec["halo_exchange_us"] > 0
    if "--dims" in extra:
        assert "py2 x px2" in rec["config"]["parallelism"]
    if "--overlap" in extra:
        assert rec["config"]["parallelism"].endswith("overlap")
        # the swapped process grid is timed too (2x1 -> 1x2), same engine path
        assert rec["stencil_alt_dims"] == "1x2" and rec["stencil_alt_dims_MLUPS"] > 0
    if n == 8:
        assert "py4 x px2" in rec["config"]["parallelism"]
        assert rec["stencil_alt_dims"] == "2x4" and rec["stencil_alt_dims_MLUPS"] > 0


def test_bench_ipc_peer_hang_fails_the_job():
    """Fault injection: rank 1 stops forever at its 3rd halo exchange
    (GMT_INJECT_HANG=1:2, gmt/watchdog.hpp).  Rank 0's exchange kernel gives
    up after GMT_WAIT_TIMEOUT_MS, the host reads the error word at its next
    synchronisation and aborts with a message naming the channel, and
    torchrun tears the job down: a non-zero exit and no JSON number."""
    p = _torchrun(2, ["--size", "1024", "--steps", "10", "--warmup", "2", "--skip-extras"], timeout=150,
                  GMT_INJECT_HANG="1:2", GMT_WAIT_TIMEOUT_MS="1000")
    assert p.returncode != 0, p.stdout + p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")], p.stdout
    assert "GMT FAULT INJECTION: rank 1" in p.stderr, p.stderr[-4000:]
    assert "timed out waiting for the peer" in p.stdout + p.stderr, (p.stdout + p.stderr)[-4000:]


def test_bench_push_corrupt_face_fails_the_job():
    """Fault injection on the inline halo: rank 1 overwrites one ghost cell
    its neighbour pushed, at the 2nd fused pass of the timed run
    (GMT_CORRUPT_PASS=1:2).  The check of the timed run sees the mismatch and
    the job fails, with the mismatch in the line."""
    p = _torchrun(2, ["--size", "4096", "--steps", "20", "--warmup", "5", "--skip-extras", "--skip-check",
                      "--no-calibrate", "--transport", "push"], timeout=200, GMT_CORRUPT_PASS="1:2")
    assert p.returncode != 0, p.stdout + p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout + p.stderr[-3000:]
    rec = json.loads(lines[0])
    assert rec["config"]["transport"] == "ipc inline halo"
    assert rec["timed_check_mismatches"] > 0 and rec["timed_check_failed"] == ["timed_check"], rec
    assert "GMT FAULT INJECTION: rank 1" in p.stderr
