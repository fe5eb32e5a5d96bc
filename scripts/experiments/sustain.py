"""Back-to-back K = 20 passes of one domain for a fixed wall time (a
sustained load for read-only SMI power / clock queries), then the clock
record of the last second.

    python scripts/experiments/sustain.py [n] [seconds]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gpu_mpi_tests_amd.engine import NativeJacobi  # noqa: E402
from gpu_mpi_tests_amd.parallel import dist as gd  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    env = gd.init(device="cuda")
    e = NativeJacobi(n, n, env, overlap=False, graph=False, tblock=20, init="random", seed=3, calibrate=True)
    e.prepare(20)
    print(f"sustain: start {n}^2 for {secs} s", flush=True)
    t0 = time.perf_counter()
    passes = 0
    while time.perf_counter() - t0 < secs:
        e.clock_reset()
        t1 = time.perf_counter()
        e.run(20 * 10)
        e.synchronize()
        dt = time.perf_counter() - t1
        passes += 10
        c = e.clock()
        print(f"t {time.perf_counter() - t0:6.2f} s  {n * n * 200 / dt / 1e6:12.1f} MLUPS  sclk {c['sclk_mhz']:7.1f} MHz",
              flush=True)
    e.close()


if __name__ == "__main__":
    main()
