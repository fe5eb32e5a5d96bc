"""One process holding BOTH RCCL communicators that every rank of a
multi-GPU bench.py run holds: torch.distributed's "nccl" (=RCCL) process
group and the native engine's own RCCL communicator (libgmt_ccl.so, a
periodic 1-rank self-exchange here).  The two share one librccl.so.1 (same
SONAME as torch's bundled copy).  Run under torch.distributed.run with one
process; prints "COEXIST OK <max diff>" on success.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_mpi_tests_amd import engine  # noqa: E402
from gpu_mpi_tests_amd.parallel import dist as gdist  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    t = torch.ones(1024, dtype=torch.float64, device=dev)
    dist.all_reduce(t)  # torch's RCCL communicator is live
    env = gdist.init(device="cuda")
    e = engine.NativeJacobi(200, 700, env, periodic=True, overlap=True, graph=False, tblock=20,
                            transport="rccl")
    try:
        assert e.transport == "rccl", e.transport
        e.run(45)
        e.synchronize()
        got = e.interior()
    finally:
        e.close()
    dist.all_reduce(t)  # and still live after the engine's communicator is gone
    torch.cuda.synchronize()
    assert float(t[0]) == 1.0
    diff = float(np.abs(got - engine.serial_jacobi(200, 700, 45, True)).max())
    dist.destroy_process_group()
    print(f"COEXIST OK {diff}", flush=True)
    sys.exit(0 if diff == 0.0 else 1)


if __name__ == "__main__":
    main()
