"""Rank pinning: every rank pins itself to one
physical core near its GPU, a distinct core per local rank, narrowing (never
widening) a launcher's binding (gmt_rt_pin_rank, gmt/numa_bind.hpp).  On the
CPU backend it is off unless GMT_PIN=1, so side-by-side test jobs do not all
land on one core."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_LIB = os.path.join(ROOT, "build", "lib-host", "libgmt.so")

CODE = ("import ctypes, os, sys; L = ctypes.CDLL(sys.argv[1]); c = ctypes.c_int(-1);"
        "L.gmt_rt_pin_rank(int(sys.argv[2]), int(sys.argv[3]), 1, ctypes.byref(c));"
        "print(c.value, ','.join(map(str, sorted(os.sched_getaffinity(0)))))")


def _pin(rank, size, **env):
    e = {k: v for k, v in os.environ.items() if k != "GMT_PIN"}
    e.update(env)
    p = subprocess.run([sys.executable, "-c", CODE, HOST_LIB, str(rank), str(size)], capture_output=True,
                       text=True, timeout=60, env=e, check=True)
    cpu, cpus = p.stdout.split()
    return int(cpu), {int(c) for c in cpus.split(",")}


def _cores():
    seen, cores = set(), []
    for c in sorted(os.sched_getaffinity(0)):
        if c in seen:
            continue
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                txt = f.read().strip()
            sib = set()
            for part in txt.split(","):
                a, _, b = part.partition("-")
                sib |= set(range(int(a), int(b or a) + 1))
        except OSError:
            sib = {c}
        seen |= sib
        cores.append(c)
    return cores


def test_host_backend_default_is_off():
    allowed = os.sched_getaffinity(0)
    cpu, got = _pin(0, 2)
    assert cpu == -1 and got == allowed


def test_pin_distinct_cores_within_the_allowed_set():
    allowed = os.sched_getaffinity(0)
    cores = _cores()
    if len(cores) < 2:
        import pytest
        pytest.skip("needs two cores")
    c0, s0 = _pin(0, 2, GMT_PIN="1")
    c1, s1 = _pin(1, 2, GMT_PIN="1")
    assert c0 in cores and c1 in cores and c0 != c1
    assert c0 in s0 and c1 in s1 and not (s0 & s1)
    assert s0 <= allowed and s1 <= allowed and len(s0) < len(allowed)
    # consecutive cores in local-rank order (one CCD, like -bind-to core)
    assert cores.index(c0) == 0 and cores.index(c1) == 1


def test_launcher_binding_is_narrowed_not_widened():
    cores = _cores()
    if len(cores) < 3:
        import pytest
        pytest.skip("needs three cores")
    keep = set(cores[1:3])  # a launcher bound this rank to two cores (first threads only)
    code = f"import os; os.sched_setaffinity(0, {sorted(keep)!r}); " + CODE.replace("import ctypes, os, sys; ", "import ctypes, sys; ")
    e = dict(os.environ, GMT_PIN="1")
    p = subprocess.run([sys.executable, "-c", "import os, ctypes, sys; " + code, HOST_LIB, "1", "2"],
                       capture_output=True, text=True, timeout=60, env=e, check=True)
    cpu, cpus = p.stdout.split()
    got = {int(c) for c in cpus.split(",")}
    assert int(cpu) == cores[2] and got == {cores[2]}
