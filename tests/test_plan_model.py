"""The temporal-blocking kernel's segment planner, on the host (CPU-only).

``build/bench/plan_model --check-bands`` plans band-first passes (row bands of
20 rows on the halo row sides, csrc/engine/jacobi.cpp band_rects) for every
built sweep count over a sweep of shares, halo masks and resident-slot counts,
and checks that every row-band segment holds at least the rows it signals:
a shorter band's output wave never counts its arrival and the pass never
signals (the round-5 hang of bench.py --overlap on at 2 ranks: 64 segments of
64 rows over 4036 left 4 rows for the last one).  The kernel now splits an
interior into segments whose lengths differ by one row at most
(csrc/kernels/jacobi5tb.hpp tb_block)."""
import os
import subprocess

from native_util import ROOT

TOOL = os.path.join(ROOT, "build", "bench", "plan_model")


def _tool():
    subprocess.run(["make", "-C", ROOT, "build/bench/plan_model"], check=True, stdout=subprocess.DEVNULL)
    return TOOL


def test_band_segments_hold_their_signalled_rows():
    p = subprocess.run([_tool(), "--check-bands"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:]
    assert "band plans: 0 violations" in p.stdout


def test_headline_plans_print():
    p = subprocess.run([_tool()], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "32768 x  32768 mask  0" in p.stdout and "workgroups on 1024 slots" in p.stdout


def test_tail_swizzle_is_a_permutation():
    """GMT_TB_EDGES_LAST's block -> tile map (csrc/kernels/jacobi5tb.hpp
    tail_swizzle): every tile exactly once, on every launch shape the
    launcher accepts it for."""
    p = subprocess.run([_tool(), "--check-swizzle"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:]
    assert " 0 of " in p.stdout


def test_shared_group_plans():
    """Shared hand-off group launches (GMT_PLAN_SH=1: four strips per
    8-wave workgroup, 920 output columns per group at K = 20, one workgroup
    per CU): the x-halo shapes the launcher gives them fit their 256 slots
    in one round where the per-strip plan does, and the 32768^2 plan runs
    several rounds with its edge segments last."""
    env = dict(os.environ, GMT_PLAN_SH="1")
    p = subprocess.run([_tool(), "8192", "8192", "15", "1024", "8192", "16384", "15", "1024",
                        "32768", "32768", "0", "1024"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = p.stdout.strip().splitlines()
    assert len(lines) == 3, p.stdout
    for ln in lines[:2]:
        wgs = int(ln.split(" workgroups on ")[0].rsplit(" ", 1)[1])
        assert "on 256 slots" in ln and 200 <= wgs <= 256, ln
    assert "edges last" in lines[2] and "on 256 slots" in lines[2], lines[2]
