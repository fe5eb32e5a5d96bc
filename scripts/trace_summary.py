#!/usr/bin/env python3
"""Summarise GMT_HOST_TRACE files (csrc/comm/transport_mpi.cpp): per run
directory and rank, the median of each host-side phase of the mpi-host
exchanges (microseconds after the exchange's start; the first exchange,
which sets up connections, is skipped).

    python scripts/trace_summary.py gpurun_out/r05_h/xport/halo_*"""
import glob
import os
import statistics
import sys

COLS = ["wait", "first_staged", "last_staged", "first_landed", "last_landed", "recvd", "end"]


def summarise(path):
    rows = []
    for ln in open(path):
        if ln.startswith("#") or not ln.strip():
            continue
        f = ln.split()
        rows.append([float(x) for x in f[2:2 + len(COLS)]])
    rows = rows[1:]
    if not rows:
        return None
    return [statistics.median(r[i] for r in rows) for i in range(len(COLS))], len(rows)


def main(argv):
    print("%-40s %5s " % ("run/rank", "n") + " ".join("%12s" % c for c in COLS))
    for d in argv:
        for f in sorted(glob.glob(os.path.join(d, "host_trace_r*.txt"))):
            r = summarise(f)
            if r:
                med, n = r
                name = os.path.basename(d.rstrip("/")) + "/" + os.path.basename(f)[11:-4]
                print("%-40s %5d " % (name, n) + " ".join("%12.1f" % v for v in med))


if __name__ == "__main__":
    main(sys.argv[1:])
