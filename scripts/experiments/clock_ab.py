"""Same-process A/B of the fused passes with and without the shader-clock
record (GMT_CLOCK=0 turns the sampled s_memtime / s_memrealtime stamps off),
alternating, and the clock each timed run ran at: does the record cost
anything, and does MLUPS track the clock?

    python scripts/experiments/clock_ab.py [n] [steps] [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gpu_mpi_tests_amd.engine import NativeJacobi  # noqa: E402
from gpu_mpi_tests_amd.parallel import dist as gd  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    env = gd.init(device="cuda")
    engines = {}
    for mode in ("on", "off"):
        os.environ["GMT_CLOCK"] = "1" if mode == "on" else "0"
        e = NativeJacobi(n, n, env, overlap=False, graph=False, tblock=20, init="random", seed=3, calibrate=True)
        e.prepare(steps)
        engines[mode] = e
    for e in engines.values():  # warm the clock up: a few seconds of passes
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            e.run(steps)
            e.synchronize()
    for rep in range(reps):
        for mode in (("on", "off") if rep % 2 == 0 else ("off", "on")):
            e = engines[mode]
            e.synchronize()
            e.clock_reset()
            t0 = time.perf_counter()
            e.run(steps)
            e.synchronize()
            dt = time.perf_counter() - t0
            c = e.clock()
            print(f"n {n} rep {rep} clock-record {mode:3s} {n * n * steps / dt / 1e6:12.1f} MLUPS "
                  f"{dt / steps * 1e3:.4f} ms/step  sclk {c['sclk_mhz']:7.1f} MHz ({c['samples']} samples)", flush=True)
    for e in engines.values():
        e.close()


if __name__ == "__main__":
    main()
