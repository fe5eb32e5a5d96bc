"""Python front end of the native Jacobi engine (``libgmt_engine.so``).

The flagship benchmark's step loop runs in C++ (``csrc/engine/jacobi.cpp``):
halo exchange over RCCL (one rank per GPU) or HIP IPC (several ranks per
GPU, or any same-node job) on a high-priority stream overlapped with the
interior sweep, both step parities captured into hipGraphs.  Python only does
the rendezvous: ``torch.distributed`` broadcasts a 128-byte id (the RCCL
unique id, or the name of the IPC transport's socket control plane), then
each ``run(k)`` is a single ctypes call that enqueues k graph replays — no
Python on the per-step critical path, which is what keeps small per-GPU
domains (strong scaling to 8 GPUs) from going launch-bound.

Transport choice (``transport="auto"``, or GMT_TRANSPORT in the environment):
RCCL when every rank has its own GPU, IPC when ranks share one (RCCL refuses
two ranks on one device; the reference's oversubscription mode,
mpi_daxpy.cc:43-54); on the CPU backend the socket emulation of RCCL, with
"ipc" selecting the memfd emulation of the IPC path.

Library selection: device ``cuda`` loads ``gpu_mpi_tests_amd/_lib`` (HIP,
gfx950); device ``cpu`` loads ``build/lib-host`` (the CPU backend, same ABI)
so the engine is testable without a GPU.  Both export SONAME ``libgmt.so``,
so one process can only hold one backend — mixing raises instead of silently
binding the wrong one.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from .parallel import dist as gdist

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
HIP_ENGINE = os.path.join(_HERE, "_lib", "libgmt_engine.so")
HOST_ENGINE = os.path.join(_ROOT, "build", "lib-host", "libgmt_engine.so")

LOCAL, RCCL, IPC = 0, 1, 2
INITS = {"analytic": 0, "random": 1}  # JacobiConfig::init
_KINDS = {"local": LOCAL, "rccl": RCCL, "ipc": IPC}
MAX_TSTEPS = 20  # GMT_TB_MAX_SWEEPS (csrc/include/gmt/kernels.h)
_libs: dict[str, ctypes.CDLL] = {}


class EngineOpts(ctypes.Structure):
    """gmt_engine_opts (csrc/include/gmt/engine.h)."""
    _fields_ = [(n, ctypes.c_int) for n in
                ("periodic", "overlap", "graph", "tsteps", "wg_waves", "seg_rows", "exact", "init",
                 "calibrate")] + [("seed", ctypes.c_int64), ("push", ctypes.c_int)]


class EngineError(RuntimeError):
    pass


def load(device: str = "cuda") -> ctypes.CDLL:
    kind = "hip" if device.startswith("cuda") else "host"
    if kind in _libs:
        return _libs[kind]
    other = "host" if kind == "hip" else "hip"
    if other in _libs:
        raise EngineError(f"the {other} engine backend is already loaded in this process; "
                          f"run the {kind} engine in a separate process")
    path = HIP_ENGINE if kind == "hip" else HOST_ENGINE
    if not os.path.exists(path):
        raise EngineError(f"{path} is missing: build it with `make lib host` "
                          "(or __graft_entry__.build())")
    if kind == "hip":
        import torch  # noqa: F401  -- torch owns the HIP runtime first (see _native.py)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    vp, i64, c_int = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.gmt_engine_unique_id.argtypes = [vp]
    lib.gmt_engine_unique_id.restype = c_int
    lib.gmt_engine_control_id.argtypes = [vp]
    lib.gmt_engine_control_id.restype = c_int
    lib.gmt_engine_comm_create.argtypes = [c_int, c_int, c_int, vp]
    lib.gmt_engine_comm_create.restype = vp
    lib.gmt_engine_comm_allreduce_sum.argtypes = [vp, vp, i64, vp]
    lib.gmt_engine_comm_allreduce_sum.restype = c_int
    lib.gmt_engine_comm_name.argtypes = [vp]
    lib.gmt_engine_comm_name.restype = ctypes.c_char_p
    lib.gmt_engine_comm_destroy.argtypes = [vp]
    lib.gmt_engine_comm_destroy.restype = None
    lib.gmt_engine_jacobi_create.argtypes = [i64, i64, c_int, c_int, c_int, c_int, c_int, vp, vp]
    lib.gmt_engine_jacobi_create.restype = vp
    lib.gmt_engine_jacobi_destroy.argtypes = [vp]
    lib.gmt_engine_jacobi_destroy.restype = None
    for name in ("gmt_engine_jacobi_sync", "gmt_engine_jacobi_exchange"):
        getattr(lib, name).argtypes = [vp]
        getattr(lib, name).restype = c_int
    lib.gmt_engine_jacobi_run.argtypes = [vp, c_int]
    lib.gmt_engine_jacobi_run.restype = c_int
    lib.gmt_engine_jacobi_residual.argtypes = [vp]
    lib.gmt_engine_jacobi_residual.restype = ctypes.c_double
    lib.gmt_engine_jacobi_info.argtypes = [vp, ctypes.POINTER(i64)]
    lib.gmt_engine_jacobi_info.restype = c_int
    lib.gmt_engine_jacobi_tb_info.argtypes = [vp, c_int, ctypes.POINTER(i64)]
    lib.gmt_engine_jacobi_tb_info.restype = c_int
    lib.gmt_engine_jacobi_plan.argtypes = [vp, c_int, ctypes.POINTER(c_int), c_int]
    lib.gmt_engine_jacobi_plan.restype = c_int
    lib.gmt_engine_jacobi_prepare.argtypes = [vp, c_int]
    lib.gmt_engine_jacobi_prepare.restype = c_int
    lib.gmt_engine_jacobi_copy_interior.argtypes = [vp, vp]
    lib.gmt_engine_jacobi_copy_interior.restype = c_int
    lib.gmt_engine_jacobi_compare.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_double)]
    lib.gmt_engine_jacobi_compare.restype = c_int
    lib.gmt_engine_jacobi_clock.argtypes = [vp, c_int, ctypes.POINTER(ctypes.c_double)]
    lib.gmt_engine_jacobi_clock.restype = c_int
    lib.gmt_engine_jacobi_stat.argtypes = [vp, c_int]
    lib.gmt_engine_jacobi_stat.restype = ctypes.c_double
    lib.gmt_engine_backend.restype = ctypes.c_char_p
    lib.gmt_engine_deriv_bench.argtypes = [i64, i64, c_int, c_int, c_int, c_int, c_int, vp, vp, c_int]
    lib.gmt_engine_deriv_bench.restype = c_int
    lib.gmt_engine_watchdog_kick.argtypes = [ctypes.c_char_p]
    lib.gmt_engine_watchdog_kick.restype = None
    lib.gmt_engine_watchdog_epitaph.argtypes = [ctypes.c_char_p, c_int]
    lib.gmt_engine_watchdog_epitaph.restype = None
    lib.gmt_engine_watchdog_timeout.argtypes = []
    lib.gmt_engine_watchdog_timeout.restype = ctypes.c_double
    # from libgmt (a dependency of the engine library: found through its handle)
    lib.gmt_jacobi5tb_group_cols.argtypes = [c_int, c_int]
    lib.gmt_jacobi5tb_group_cols.restype = i64
    got = lib.gmt_engine_backend().decode()
    if got != kind:
        raise EngineError(f"{path} bound to the {got} runtime, expected {kind} "
                          "(another libgmt.so is already loaded in this process)")
    _libs[kind] = lib
    return lib


def watchdog_kick(phase: str, device: str = "cpu") -> None:
    """Marks progress for the engine's hang watchdog (GMT_TIMEOUT seconds of
    no progress end the process with status 124 and a line naming the rank
    and the last phase; gmt/watchdog.hpp).  A no-op until an engine entry
    point has armed it."""
    load(device).gmt_engine_watchdog_kick(phase.encode()[:95])


def watchdog_epitaph(text: "str | None", code: int = 0, device: str = "cpu") -> None:
    """Last words for the hang watchdog: if it fires, ``text`` (a JSON object)
    is written to stdout with a "watchdog" field naming the stalled rank and
    phase, and the process exits with ``code`` instead of 124 ("" exits
    silently; None restores the default).  bench.py registers its result
    line once the headline is measured, so an extra that hangs cannot lose it."""
    load(device).gmt_engine_watchdog_epitaph(None if text is None else text.encode(), int(code))


def watchdog_timeout(device: str = "cpu") -> float:
    """The armed watchdog's timeout in seconds (0: not armed)."""
    return float(load(device).gmt_engine_watchdog_timeout())


def group_cols(sweeps: int, wg_waves: int = 0, device: str = "cpu") -> int:
    """Output columns one workgroup of the fused K-sweep kernel covers: the
    width of the W/E bands of a band-first (overlapped) pass."""
    return int(load(device).gmt_jacobi5tb_group_cols(int(sweeps), int(wg_waves)))


class _StdoutToStderr:
    """RCCL prints its init banner ("RCCL version : ...") on the process's
    C stdout; bench.py's driver contract is ONE JSON line on stdout, so
    communicator creation runs with fd 1 pointed at stderr."""

    def __enter__(self):
        import sys
        sys.stdout.flush()
        self._libc = ctypes.CDLL(None)
        self._libc.fflush(None)
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        import sys
        self._libc.fflush(None)
        sys.stdout.flush()
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


def _broadcast_id(lib, env, kind: int) -> bytes:
    """Rank 0 creates the transport's 128-byte id, every rank gets it."""
    buf = ctypes.create_string_buffer(128)
    if env.rank == 0:
        err = (lib.gmt_engine_unique_id if kind == RCCL else lib.gmt_engine_control_id)(buf)
        if err:
            raise EngineError(f"transport id failed: {err}")
    obj = [bytes(buf.raw) if env.rank == 0 else None]
    if env.world_size > 1:
        torch.distributed.broadcast_object_list(obj, src=0, group=env.host_group)
    return obj[0]


def resolve_transport(env, transport: str = "auto") -> str:
    """auto -> rccl with one rank per GPU, ipc when ranks share a GPU; local
    for one rank.  GMT_ENGINE_TRANSPORT (rccl|ipc) overrides auto; so does
    GMT_TRANSPORT, the native apps' variable, when it names a transport the
    engine has (its other values — mpi-host, mpi-direct — are the apps' own
    and are ignored here with a warning)."""
    if transport not in ("auto", "local", "rccl", "ipc"):
        raise ValueError(f"transport must be auto, local, rccl or ipc, got {transport!r}")
    if transport == "auto":
        eng = os.environ.get("GMT_ENGINE_TRANSPORT", "").strip().lower()
        if eng:
            if eng not in ("auto", "rccl", "ipc"):
                raise ValueError(f"GMT_ENGINE_TRANSPORT must be auto, rccl or ipc, got {eng!r}")
            transport = eng
        else:
            app = os.environ.get("GMT_TRANSPORT", "").strip().lower()
            if app in ("rccl", "ipc"):
                transport = app
            elif app not in ("", "auto"):
                import warnings
                warnings.warn(f"GMT_TRANSPORT={app!r} is a native-app transport the engine does not have; "
                              "the engine picks its own (set GMT_ENGINE_TRANSPORT to choose)", stacklevel=2)
    if transport == "auto":
        if env.world_size == 1:
            return "local"
        return "ipc" if env.is_gpu and env.ranks_per_device > 1 else "rccl"
    if transport == "local" and env.world_size != 1:
        raise ValueError("transport 'local' needs world size 1")
    if transport == "rccl" and env.is_gpu and env.ranks_per_device > 1:
        raise ValueError(f"RCCL needs one rank per GPU ({env.ranks_per_device} ranks share one): use ipc")
    return transport


def transport_label(kind: str, env) -> str:
    """Name in reports: the CPU backend's emulations carry a -host suffix."""
    return kind if env.is_gpu or kind == "local" else f"{kind}-host"


def _transport_args(lib, env, transport: str):
    kind = _KINDS[resolve_transport(env, transport)]
    if kind == LOCAL:
        return kind, None
    return kind, ctypes.create_string_buffer(_broadcast_id(lib, env, kind), 128)


class Comm:
    """A bare communicator on the engine's transports (device collectives
    outside the solver: bench.py's DAXPY partial-sum all-reduce)."""

    def __init__(self, env=None, transport: str = "auto"):
        self.env = env or gdist.get()
        self.lib = load("cuda" if self.env.is_gpu else "cpu")
        self.kind = resolve_transport(self.env, transport)
        k, cid = _transport_args(self.lib, self.env, self.kind)
        with _StdoutToStderr():
            self.h = self.lib.gmt_engine_comm_create(self.env.rank, self.env.world_size, k, cid)
        if not self.h:
            raise EngineError("gmt_engine_comm_create failed")
        self.name = transport_label(self.lib.gmt_engine_comm_name(self.h).decode(), self.env)

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks of a contiguous float64 tensor on this rank's device."""
        if t.dtype != torch.float64 or not t.is_contiguous():
            raise ValueError("allreduce_sum_ needs a contiguous float64 tensor")
        if (t.device.type == "cuda") != self.env.is_gpu:
            raise ValueError(f"tensor on {t.device}, communicator on {self.env.device}")
        stream = torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else None
        err = self.lib.gmt_engine_comm_allreduce_sum(self.h, t.data_ptr(), t.numel(), stream)
        if err:
            raise EngineError(f"all-reduce failed: {err}")
        return t

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.gmt_engine_comm_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


class NativeJacobi:
    """Distributed 2-D Jacobi (fp64) on the native engine: one rank per GPU
    (RCCL) or several ranks per GPU (IPC)."""

    def __init__(self, ny: int, nx: int, env: "gdist.DistEnv | None" = None,
                 dims: tuple[int, int] | None = None, periodic: bool = False,
                 overlap: "bool | str" = True, graph: bool = True,
                 tblock: bool | int = False, wg_waves: int = 0, seg_rows: int = 0, exact: int = -1,
                 transport: str = "auto", init: str = "analytic", seed: int = 0, calibrate: bool = False,
                 push: bool = False):
        """push: the fused passes exchange their halo inline (each pass stores
        its output faces straight into the neighbours' ghost cells over IPC
        mappings, then one hand-over launch; gmt/jacobi.hpp JacobiConfig::push).
        Needs the IPC transport when a neighbour is another rank; silently the
        transport's exchange when the share is too small (``push_active``)."""
        from .parallel.decomp import choose_dims

        self.env = env or gdist.get()
        e = self.env
        self.device = "cuda" if e.is_gpu else "cpu"
        self.lib = load(self.device)
        py, px = dims if dims else choose_dims(e.world_size, ny, nx)
        if py * px != e.world_size:
            raise ValueError(f"process grid {py}x{px} != world size {e.world_size}")
        self.ny_g, self.nx_g, self.py, self.px = ny, nx, py, px
        kind = resolve_transport(e, transport)
        if e.world_size == 1 and kind in ("rccl", "ipc"):
            # a 1-rank communicator: a periodic domain exchanges its halo with
            # itself through the transport (latency measurements)
            k = _KINDS[kind]
            cid = ctypes.create_string_buffer(_broadcast_id(self.lib, e, k), 128)
            transport = k
        else:
            # GPU: RCCL over xGMI or HIP IPC.  CPU: the host backend's
            # emulations of the same semantics (RCCL over Unix sockets,
            # csrc/host/ccl_host.cpp; IPC over memfd-shared memory), so the
            # multi-rank engine path runs and is checked without GPUs.
            transport, cid = _transport_args(self.lib, e, kind)
        ks = 1 if not tblock else (2 if tblock is True else int(tblock))
        if not 1 <= ks <= MAX_TSTEPS:
            raise ValueError(f"tblock: sweeps per fused pass must be 1..{MAX_TSTEPS}, got {ks}")
        # overlap: True / False / "auto" (time both once, every rank keeps the faster)
        auto = overlap == "auto"
        if init not in INITS:
            raise ValueError(f"init must be one of {sorted(INITS)}, got {init!r}")
        if not 0 <= int(seed) < 1 << 53:
            raise ValueError("seed must be in [0, 2^53)")
        self.init, self.seed = init, int(seed)
        opts = EngineOpts(periodic=int(bool(periodic)), overlap=2 if auto else int(bool(overlap)),
                          graph=int(bool(graph)), tsteps=ks, wg_waves=int(wg_waves),
                          seg_rows=int(seg_rows), exact=int(exact), init=INITS[init],
                          calibrate=int(bool(calibrate)), seed=int(seed), push=int(bool(push)))
        with _StdoutToStderr():
            self.h = self.lib.gmt_engine_jacobi_create(ny, nx, py, px, e.rank, e.world_size, transport,
                                                       cid, ctypes.byref(opts))
        if not self.h:
            raise EngineError("gmt_engine_jacobi_create failed")
        info = (ctypes.c_int64 * 16)()
        self.lib.gmt_engine_jacobi_info(self.h, info)
        (self.nx, self.ny, self.off_x, self.off_y, self.halo_bytes, self.halo_msgs,
         graph_on, overlap_on, _, _, tb, t_ov, t_ser, exact_on, band_on, push_on) = list(info)
        self.push_active = bool(push_on)
        # overlapped fused passes run band-first (boundary bands signal, the
        # output halo travels under the interior)
        self.band_first = bool(band_on)
        self.exact = bool(exact_on)
        # overlap="auto": measured seconds per fused pass {overlap, serial} (mean over ranks)
        self.tuned = {"overlap_s": t_ov / 1e9, "serial_s": t_ser / 1e9} if auto and t_ov else None
        self.tsteps = int(tb)
        self.tblock = self.tsteps > 1
        self.graph = bool(graph_on)
        self.overlap = bool(overlap_on)
        self.transport = transport_label(kind, e)

    # ------------------------------------------------------------------
    def run(self, steps: int) -> None:
        self.lib.gmt_engine_jacobi_run(self.h, int(steps))

    def step(self) -> None:
        self.run(1)

    def plan(self, steps: int) -> list[int]:
        """Sweeps per fused pass, in launch order, that ``run(steps)`` enqueues."""
        buf = (ctypes.c_int * max(1, steps))()
        n = self.lib.gmt_engine_jacobi_plan(self.h, int(steps), buf, max(1, steps))
        return list(buf[:n])

    def prepare(self, steps: int) -> None:
        """One pass of every pass type ``run(steps)`` uses, then the initial field again."""
        self.lib.gmt_engine_jacobi_prepare(self.h, int(steps))

    def synchronize(self) -> None:
        self.lib.gmt_engine_jacobi_sync(self.h)

    @property
    def max_abs_u0(self) -> float:
        """max |u| of the initial field over all ranks (measured on the device;
        drives the scaled-level exactness guard)."""
        return float(self.lib.gmt_engine_jacobi_stat(self.h, 0))

    def pass_cost_ms(self) -> dict:
        """A full tsteps pass: measured by a calibrated prepare() (0 before) and
        the built-in table's estimate for this share."""
        return {"measured": round(float(self.lib.gmt_engine_jacobi_stat(self.h, 1)), 4),
                "table": round(float(self.lib.gmt_engine_jacobi_stat(self.h, 2)), 4)}

    def exchange(self) -> None:
        self.lib.gmt_engine_jacobi_exchange(self.h)

    def residual(self) -> float:
        return float(self.lib.gmt_engine_jacobi_residual(self.h))

    def interior(self) -> np.ndarray:
        out = np.empty((self.ny, self.nx), dtype=np.float64)
        self.lib.gmt_engine_jacobi_copy_interior(self.h, out.ctypes.data)
        return out

    def compare(self, other: "NativeJacobi") -> tuple[float, int]:
        """Bitwise comparison of this engine's current interior with another
        engine's (same global problem and process grid), on the device:
        (max |diff| over ranks, elements whose bits differ over ranks).
        Collective: every rank calls it."""
        out = (ctypes.c_double * 2)()
        if self.lib.gmt_engine_jacobi_compare(self.h, other.h, out):
            raise EngineError("gmt_engine_jacobi_compare failed")
        return float(out[0]), int(out[1])

    def tb_launch(self, k: int) -> dict:
        """The launch shape of this rank's one-rect k-sweep pass
        (gmt_jacobi5tb_plan, nothing launched): workgroups, resident slots,
        threads per workgroup, segment rows and count, VGPRs; ``shape`` names
        it — for two-stage strips 128 threads are one strip per workgroup,
        256 two stage-major strips, 512 a shared hand-off group (default
        wg_waves) — csrc/kernels/jacobi5tb.hpp launch_tb / sh_launch."""
        out = (ctypes.c_int64 * 6)()
        rc = self.lib.gmt_engine_jacobi_tb_info(self.h, int(k), out)
        if rc != 0:
            return {"error": int(rc)}
        keys = ("workgroups", "resident", "threads", "seg_rows", "segments", "vgprs")
        d = dict(zip(keys, (int(v) for v in out)))
        if k > 10 and d["threads"] in (128, 256, 512):
            d["shape"] = {128: "one two-stage strip per workgroup",
                          256: "two two-stage strips per workgroup, stage-major waves (a shared "
                               "hand-off pair unless push / GMT_TB_SHARED=0)",
                          512: "shared hand-off group: four strips, stage-major waves"}[d["threads"]]
        return d

    def clock_reset(self) -> None:
        """Zero the fused passes' shader-clock record (stream ordered)."""
        self.lib.gmt_engine_jacobi_clock(self.h, 1, None)

    def clock(self) -> dict:
        """The clock the fused passes ran at since clock_reset(): sampled
        waves' s_memtime / s_memrealtime deltas (gmt_tb_opts.clock).  MHz is
        0 on the CPU backend or without samples (GMT_CLOCK=0)."""
        out = (ctypes.c_double * 3)()
        self.lib.gmt_engine_jacobi_clock(self.h, 0, out)
        return {"sclk_mhz": round(out[0], 1), "samples": int(out[1]), "sampled_s": round(out[2], 6)}

    @property
    def points(self) -> int:
        return self.ny_g * self.nx_g

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.gmt_engine_jacobi_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


def deriv_bench(n_local: int = 1024, n_other: int = 512 * 1024, n_iter: int = 100,
                n_warmup: int = 5, env: "gdist.DistEnv | None" = None, transport: str = "auto",
                check: bool = False) -> dict:
    """The reference's main benchmark on the native engine (one rank per GPU,
    RCCL): ``mpi_stencil2d_gt``'s test_deriv for dim 0 and dim 1 (2-deep
    ghost faces of ``n_other`` values per neighbour — 8 MiB at the reference
    default — exchanged, then the derivative kernel, ``n_iter`` times) and
    test_sum (in-place all-reduce of 1024 doubles).  Returns this rank's
    per-exchange seconds (median/mean/min/max), bytes sent per exchange,
    err_norm, and the all-reduce median seconds.  Collective: every rank calls it.
    Transport as NativeJacobi (RCCL, IPC when ranks share a GPU).  ``check``: the
    ghost rows are compared with the analytic field after every exchange
    (``bad_ghosts`` per dim; the exchanges stay timed alone)."""
    e = env or gdist.get()
    lib = load("cuda" if e.is_gpu else "cpu")
    transport, cid = _transport_args(lib, e, transport)
    out = (ctypes.c_double * 18)()
    with _StdoutToStderr():
        err = lib.gmt_engine_deriv_bench(int(n_local), int(n_other), int(n_iter), int(n_warmup), e.rank,
                                         e.world_size, transport, cid, out, int(bool(check)))
    if err:
        raise EngineError(f"gmt_engine_deriv_bench failed: {err}")
    v = list(out)
    res = {}
    for d in (0, 1):
        o = v[6 * d:6 * d + 6]
        res[f"dim{d}"] = dict(median_s=o[0], mean_s=o[1], min_s=o[2], max_s=o[3], bytes=int(o[4]),
                              err_norm=o[5], exact_norm=v[14 + d], bad_ghosts=int(v[16 + d]))
    res["allreduce_median_s"] = v[12]
    res["allreduce_max_rel_err"] = v[13]
    res["transport"] = transport_label({LOCAL: "local", RCCL: "rccl", IPC: "ipc"}[transport], e)
    return res


def lattice_uniform(gx: np.ndarray, gy: np.ndarray, seed: int) -> np.ndarray:
    """uniform [0, 1) of integer lattice points: the same splitmix64 hash as
    gmt_fill_poly mode 5 (csrc/kernels/reduce.hip lattice_uniform), bitwise."""
    u64 = np.uint64
    gx = np.asarray(gx, dtype=np.int64) + (1 << 30)
    gy = np.asarray(gy, dtype=np.int64) + (1 << 30)
    k = (gy.astype(u64) << u64(32)) ^ gx.astype(u64)
    k = k ^ u64(seed)
    k = k + u64(0x9E3779B97F4A7C15)
    k = (k ^ (k >> u64(30))) * u64(0xBF58476D1CE4E5B9)
    k = (k ^ (k >> u64(27))) * u64(0x94D049BB133111EB)
    k = k ^ (k >> u64(31))
    return (k >> u64(11)).astype(np.float64) * 2.0 ** -53


def initial_field(ny: int, nx: int, init: str = "analytic", seed: int = 0) -> np.ndarray:
    """The engine's initial field with its ghost ring, (ny+2) x (nx+2),
    global lattice index -1..n (gmt_fill_poly mode 4 / 5)."""
    if init == "random":
        gx = np.arange(-1, nx + 1, dtype=np.int64)[None, :]
        gy = np.arange(-1, ny + 1, dtype=np.int64)[:, None]
        return lattice_uniform(np.broadcast_to(gx, (ny + 2, nx + 2)), np.broadcast_to(gy, (ny + 2, nx + 2)), seed)
    if init != "analytic":
        raise ValueError(f"init must be analytic or random, got {init!r}")
    h = 1.0 / (max(ny, nx) + 1)
    x = (np.arange(nx + 2, dtype=np.float64) - 1.0) * h
    y = (np.arange(ny + 2, dtype=np.float64) - 1.0) * h
    return (x[None, :] * x[None, :] * x[None, :]) + (y[:, None] * y[:, None])


def serial_jacobi(ny: int, nx: int, steps: int, periodic: bool = False, init: str = "analytic",
                  seed: int = 0) -> np.ndarray:
    """NumPy reference of exactly the engine's problem (init, boundary, update):
    bitwise — the engine fills x^3 + y^2 on the same integer lattice with the
    same operation order (gmt_fill_poly mode 4), or the same hashed random
    field (mode 5), and sweeps in the same order."""
    u = initial_field(ny, nx, init, seed)
    un = u.copy()
    for _ in range(steps):
        if periodic:
            u[1:-1, 0] = u[1:-1, -2]
            u[1:-1, -1] = u[1:-1, 1]
            u[0, 1:-1] = u[-2, 1:-1]
            u[-1, 1:-1] = u[1, 1:-1]
        un[1:-1, 1:-1] = 0.25 * ((u[1:-1, :-2] + u[1:-1, 2:]) + (u[:-2, 1:-1] + u[2:, 1:-1]))
        u, un = un, u
    return u[1:-1, 1:-1].copy()
