"""Same-process A/B of the K = 20 pass on random vs analytic (smooth) field
data: is the pass power-bound on data-dependent switching?  One rank,
Dirichlet boundary, the engine's own plan; alternating, three reps.

    python scripts/experiments/init_ab.py [n] [steps]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from gpu_mpi_tests_amd.engine import NativeJacobi  # noqa: E402
from gpu_mpi_tests_amd.parallel import dist as gd  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    env = gd.init(device="cuda")
    engines = {}
    for init in ("random", "analytic"):
        e = NativeJacobi(n, n, env, overlap=False, graph=False, tblock=20, init=init, seed=3)
        e.prepare(steps)
        engines[init] = e
    for rep in range(3):
        for init, e in engines.items():
            e.run(steps)  # warm
            e.synchronize()
            t0 = time.perf_counter()
            e.run(steps)
            e.synchronize()
            dt = time.perf_counter() - t0
            print(f"n {n} rep {rep} init {init:8s} {n * n * steps / dt / 1e6:12.1f} MLUPS  {dt / steps * 1e3:.4f} ms/step",
                  flush=True)
    for e in engines.values():
        e.close()


if __name__ == "__main__":
    main()
