#!/usr/bin/env python3
"""Per-workgroup timeline of one K-sweep pass (GMT_TB_WG_TRACE builds,
csrc/kernels/jacobi5tb.hpp; scripts/experiments/gpu_r05_l.sh): workgroup
durations by tile kind (edge segments, boundary strip groups, interior), the
cost per step of each kind relative to interior tiles, and per-XCD finish
times against the whole pass.

    python scripts/wg_timeline.py gpurun_out/r05_l/wg_*.txt*"""
import collections
import statistics
import sys

U, LAG = 19, 2  # K = 20 strip: unrolled steps per block, output-stage lag


def parse(path):
    hdr, rows = {}, []
    for ln in open(path):
        if ln.startswith("# K"):
            f = ln[2:].split()
            i = 0
            while i < len(f):
                key = f[i]
                if key == "rect0":
                    hdr[key] = [int(x) for x in f[i + 1:i + 5]]
                    i += 5
                else:
                    hdr[key] = int(f[i + 1])
                    i += 2
        elif not ln.startswith("#") and ln.strip():
            b, t, s, e, hw, xcc = (int(x) for x in ln.split())
            rows.append((b, t, s, e, hw, xcc))
    return hdr, rows


def kind_of(h, t):
    ngroups = (h["nstrip"] + h["nw"] - 1) // h["nw"]
    nedge = (h["e0"] > 0) + (h["e1"] > 0)
    nbnd = 2 if ngroups > 1 else 1
    n_ed = nedge * ngroups
    n_bd = h["nmid_b"] * nbnd
    if t < n_ed:
        gi = t % ngroups
        edge = 0 if (t // ngroups == 0 and h["e0"] > 0) else 1
        rows = h["e0"] if edge == 0 else h["e1"]
        return ("edge-bnd" if gi in (0, ngroups - 1) else "edge"), rows
    if t < n_ed + n_bd:
        return "bnd", h["lmid_b"]
    return "mid", h["lmid"]


def steps(rows, k):
    return (rows + 2 * k + LAG + U - 1) // U * U


def main(paths):
    for p in paths:
        h, rows = parse(p)
        if not rows:
            continue
        k = h["K"]
        t0 = min(r[2] for r in rows)
        t1 = max(r[3] for r in rows)
        span = (t1 - t0) / 100.0  # us (s_memrealtime: 100 MHz)
        by = collections.defaultdict(list)
        for b, t, s, e, hw, xcc in rows:
            kind, r = kind_of(h, t)
            by[kind].append(((e - s) / 100.0, r))
        print("%s: %d workgroups, pass %.1f us, plan e %d/%d mid %d x %d bnd %d x %d, slots %d" % (
            p, len(rows), span, h["e0"], h["e1"], h["nmid"], h["lmid"], h["nmid_b"], h["lmid_b"], h["per_cu"]))
        mid_ps = None
        if by.get("mid"):
            mid_ps = statistics.median(d / steps(r, k) for d, r in by["mid"])
        for kind in ("edge", "edge-bnd", "bnd", "mid"):
            v = by.get(kind)
            if not v:
                continue
            ps = statistics.median(d / steps(r, k) for d, r in v)
            print("   %-8s %5d  rows %5d  median %8.1f us  min %8.1f  max %8.1f  us/step %.3f  x%.2f of mid" % (
                kind, len(v), v[0][1], statistics.median(d for d, _ in v), min(d for d, _ in v),
                max(d for d, _ in v), ps, ps / mid_ps if mid_ps else float("nan")))
        fin = collections.defaultdict(float)
        busy = collections.defaultdict(float)
        for b, t, s, e, hw, xcc in rows:
            fin[xcc] = max(fin[xcc], (e - t0) / 100.0)
            busy[xcc] += (e - s) / 100.0
        print("   per XCD: finish (us) " + " ".join("%d:%.0f" % (x, fin[x]) for x in sorted(fin)))
        print("   per XCD: busy / slot (us) " + " ".join("%d:%.0f" % (x, busy[x] / (h["per_cu"] / 8)) for x in sorted(busy)))


if __name__ == "__main__":
    main(sys.argv[1:])
