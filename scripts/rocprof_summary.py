#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (``*_results.db``) as markdown.

Usage: python scripts/rocprof_summary.py <results.db | *_kernel_stats.csv> [--bytes KERNEL_SUBSTR=BYTES ...] [-o out.md]

``--bytes`` attaches a known byte count per dispatch to kernels whose name
contains the substring, so the table shows the achieved bandwidth (GB/s) next
to the HBM3E roofline (~6.3 TB/s measured stream rate on MI355X).
"""
from __future__ import annotations

import argparse
import csv
import re
import sqlite3


def short(name: str, width: int = 90) -> str:
    s = re.sub(r"\(.*", "", name) if not name.startswith("void at::") else name
    s = s.replace("void ", "")
    if s.startswith("at::native::"):
        m = re.search(r"at::native::(\w+)", s)
        s = "torch:" + (m.group(1) if m else "elementwise")
        if "FillFunctor" in name:
            s += "<fill>"
        elif "direct_copy" in name:
            s += "<copy>"
        elif "uniform" in name:
            s += "<uniform>"
    return s[:width]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--bytes", action="append", default=[], help="SUBSTR=BYTES per dispatch")
    ap.add_argument("-o", "--out")
    ap.add_argument("--title", default="rocprofv3 kernel statistics")
    a = ap.parse_args(argv)
    nbytes = []
    for kv in a.bytes:
        k, v = kv.rsplit("=", 1)
        nbytes.append((k, float(eval(v, {"__builtins__": {}}))))  # simple arithmetic only
    if a.db.endswith(".csv"):  # rocprofv3 --stats --output-format csv (durations in ns)
        with open(a.db) as f:
            rows = [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                     float(r["AverageNs"]) / 1e3, float(r["Percentage"])) for r in csv.DictReader(f)]
    else:
        c = sqlite3.connect(a.db)
        rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    out = [f"# {a.title}", "", f"source: `{a.db}` (rocprofv3 --kernel-trace --stats)", "",
           "| kernel | calls | total µs | avg µs | % | GB/s (known bytes) |", "|---|---|---|---|---|---|"]
    for name, calls, tot, avg, pct in rows:
        bw = ""
        for k, b in nbytes:
            if k in name:
                bw = f"{b / (avg * 1e-6) / 1e9:,.0f}"
        out.append(f"| `{short(name)}` | {calls} | {tot:,.1f} | {avg:,.2f} | {pct:.1f} | {bw} |")
    txt = "\n".join(out) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
