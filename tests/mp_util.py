"""Multi-process (gloo, CPU) launcher for distributed tests — the CPU analogue of
the reference's oversubscribed `mpirun -np N` runs."""
import os
import traceback

import torch.multiprocessing as mp


def _entry(rank, world, port, fn, args, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    from gpu_mpi_tests_amd.parallel import dist as gdist

    try:
        env = gdist.init(device="cpu")
        res = fn(env, *args)
        q.put((rank, "ok", res))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        gdist.shutdown()


def run_dist(fn, world, port, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, status, val = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{val}")
            out[rank] = val
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [out[r] for r in range(world)]
