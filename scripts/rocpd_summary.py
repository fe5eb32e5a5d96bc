#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 rocpd SQLite database (the default
output format of this ROCm's rocprofv3): one CSV row per kernel name with
calls, total / mean / min / max duration (ns), VGPRs, scratch and LDS bytes.

  scripts/rocpd_summary.py gpurun_out/x/prof/bench_results.db > profiles/x/kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), max(vgpr_count), "
        "max(accum_vgpr_count), max(scratch_size), max(lds_size) from kernels group by name "
        "order by sum(duration) desc").fetchall()
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_ns", "mean_ns", "min_ns", "max_ns", "vgpr", "agpr", "scratch", "lds"])
    for r in rows:
        w.writerow([r[0], r[1], int(r[2]), round(r[3], 1), int(r[4]), int(r[5]), r[6], r[7], r[8], r[9]])


if __name__ == "__main__":
    main()
