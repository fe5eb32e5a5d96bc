#!/usr/bin/env python3
"""Per-kernel mean duration and busy/idle accounting of a rocprofv3 kernel
trace (``*_kernel_trace.csv``), over the last N dispatches.

    python scripts/trace_passes.py gpurun_out/x/p/per_kernel_trace.csv [--last 200]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=200)
    ap.add_argument("--skip-tail", type=int, default=6, help="drop the final N dispatches (residual etc.)")
    ap.add_argument("--timeline", default="", help="also list every dispatch whose name contains this "
                    "(duration, gap to the previous one of them): clock drift over back-to-back passes")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if a.skip_tail:
        rows = rows[:-a.skip_tail]
    rows = rows[-a.last:]
    t0 = int(rows[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    agg = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = f'{name} grid={r["Grid_Size_X"]} q{r["Queue_Id"]}'
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"window {(t1 - t0) / 1e3:.1f} us, {len(rows)} dispatches")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):5d} x {sum(v) / len(v):9.2f} us = {sum(v):10.1f} us  {k}")
    # union of busy intervals (any queue)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    busy, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
    if a.timeline:
        prev = None
        for r in rows:
            if a.timeline not in r["Kernel_Name"]:
                continue
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s0 - prev) / 1e3 if prev is not None else 0.0
            print(f"  {(e0 - s0) / 1e3:9.1f} us  gap {gap:8.1f} us  {r['Kernel_Name'].split('(')[0].replace('void ', '')}")
            prev = e0


if __name__ == "__main__":
    main()
