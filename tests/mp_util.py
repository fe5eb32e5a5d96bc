"""Multi-process (gloo, CPU) launcher for distributed tests — the CPU analogue of
the reference's oversubscribed `mpirun -np N` runs.

A rank that dies without reporting (a native abort, a signal, the OOM killer)
is named with its exit code or signal and the tail of its own stderr, which
each child writes to a file of its own (an exception inside the rank is
reported with its traceback, as before)."""
import os
import queue
import signal
import tempfile
import time
import traceback

import torch.multiprocessing as mp


def _plain(v):
    """Tensors -> NumPy copies.  torch.multiprocessing pickles a tensor as a
    shared-memory handle the receiver fetches from the SENDER's fd server: a
    rank that exits right after posting leaves the parent an EOFError (the
    round-3 '-n 8' failure), so results travel by value."""
    import torch

    if isinstance(v, torch.Tensor):
        return _ByValue(v.detach().cpu().numpy().copy())
    if isinstance(v, (list, tuple)):
        return type(v)(_plain(x) for x in v)
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    return v


class _ByValue:
    def __init__(self, a):
        self.a = a


def _restore(v):
    import torch

    if isinstance(v, _ByValue):
        return torch.from_numpy(v.a)
    if isinstance(v, (list, tuple)):
        return type(v)(_restore(x) for x in v)
    if isinstance(v, dict):
        return {k: _restore(x) for k, x in v.items()}
    return v


def _entry(rank, world, port, fn, args, q, errpath):
    # this rank's stderr (Python and native) goes to its own file
    fd = os.open(errpath, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    os.dup2(fd, 2)
    os.close(fd)
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    from gpu_mpi_tests_amd.parallel import dist as gdist

    try:
        env = gdist.init(device="cpu")
        res = fn(env, *args)
        q.put((rank, "ok", _plain(res)))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        gdist.shutdown()


def _tail(path, n=40):
    try:
        with open(path, errors="replace") as f:
            return "".join(f.readlines()[-n:])
    except OSError:
        return "(no stderr file)"


def _how(code):
    if code is None:
        return "still running"
    if code < 0:
        try:
            return f"killed by signal {signal.Signals(-code).name}"
        except ValueError:
            return f"killed by signal {-code}"
    return f"exit code {code}"


def run_dist(fn, world, port, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tmp = tempfile.mkdtemp(prefix="gmt_mp_")
    errs = [os.path.join(tmp, f"rank{r}.err") for r in range(world)]
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, errs[r])) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    deadline = time.monotonic() + timeout
    try:
        while len(out) < world:
            try:
                rank, status, val = q.get(timeout=0.5)
            except queue.Empty:
                # a rank that is gone without having posted a result died
                for r, p in enumerate(procs):
                    if r not in out and p.exitcode is not None:
                        # its result may still be in the pipe: one more look
                        try:
                            rank, status, val = q.get(timeout=2.0)
                            break
                        except queue.Empty:
                            raise AssertionError(f"rank {r} of {world} died ({_how(p.exitcode)}) without a "
                                                 f"result; its stderr:\n{_tail(errs[r])}") from None
                else:
                    if time.monotonic() > deadline:
                        alive = [r for r, p in enumerate(procs) if r not in out and p.is_alive()]
                        raise AssertionError(f"ranks {alive} of {world} gave no result within {timeout} s; "
                                             f"stderr of rank {alive[0] if alive else 0}:\n"
                                             f"{_tail(errs[alive[0] if alive else 0])}") from None
                    continue
            except EOFError:
                dead = [(r, _how(p.exitcode)) for r, p in enumerate(procs) if p.exitcode not in (None, 0)]
                raise AssertionError(f"result queue closed; dead ranks {dead}; stderr of rank "
                                     f"{dead[0][0] if dead else 0}:\n{_tail(errs[dead[0][0] if dead else 0])}") from None
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{val}\nits stderr:\n{_tail(errs[rank])}")
            out[rank] = _restore(val)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join(timeout=5)
        for e in errs:
            try:
                os.unlink(e)
            except OSError:
                pass
        try:
            os.rmdir(tmp)
        except OSError:
            pass
    return [out[r] for r in range(world)]
