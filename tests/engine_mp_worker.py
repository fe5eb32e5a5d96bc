"""torchrun worker: the native Jacobi engine at world_size ranks (CPU backend,
RCCL semantics over the host emulation) vs the serial NumPy reference.
Rank 0 prints one JSON line.  Used by tests/test_engine_cpu.py."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gpu_mpi_tests_amd import engine  # noqa: E402
from gpu_mpi_tests_amd.parallel import dist as gd  # noqa: E402


def main():
    ny, nx, steps, periodic, overlap, tblock = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]),
                                                sys.argv[4] == "1", sys.argv[5] == "1", int(sys.argv[6]))
    dims = tuple(int(v) for v in sys.argv[7].split("x")) if len(sys.argv) > 7 else None
    env = gd.init(device=os.environ.get("GMT_TEST_DEVICE", "cpu"))
    e = engine.NativeJacobi(ny, nx, env, dims=dims, periodic=periodic, overlap=overlap,
                            graph=os.environ.get("GMT_TEST_GRAPH", "1") == "1", tblock=tblock,
                            push=os.environ.get("GMT_TEST_PUSH", "0") == "1")
    e.run(steps)
    e.synchronize()
    e.exchange()  # a blocking exchange on its own (bench.py's latency probe)
    part = (e.off_y, e.off_x, e.interior())
    parts = [None] * env.world_size
    dist.all_gather_object(parts, part, group=env.host_group)
    resid = e.residual()  # one more sweep + all-reduce: identical on every rank
    resids = [None] * env.world_size
    dist.all_gather_object(resids, resid, group=env.host_group)
    if env.rank == 0:
        full = np.full((ny, nx), np.nan)
        for oy, ox, a in parts:
            full[oy:oy + a.shape[0], ox:ox + a.shape[1]] = a
        ref = engine.serial_jacobi(ny, nx, steps, periodic)
        bad = np.argwhere(np.abs(full - ref) > 0)
        print(json.dumps(dict(diff=float(np.abs(full - ref).max()), transport=e.transport, nbad=int(len(bad)),
                              first_bad=bad[:4].tolist(), overlap=e.overlap, band_first=e.band_first,
                              dims=[e.py, e.px], tsteps=e.tsteps, halo=e.halo_bytes, push=e.push_active,
                              resid_same=len(set(resids)) == 1)), flush=True)
    e.close()
    gd.shutdown()


if __name__ == "__main__":
    main()
