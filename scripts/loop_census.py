#!/usr/bin/env python3
"""Instruction census of the loops of one kernel in a gfx950 .s file
(hipcc --cuda-device-only -S): for every backward branch, the instruction
classes of the blocks between its target label and the branch.

  scripts/loop_census.py kf.s '_ZN3gmt2tb16jacobi5tb_kernelILi20ELb0ELb0E'
"""
import re
import sys
from collections import Counter

CLASSES = [
    ("dadd", r"^v_add_f64"), ("dmul", r"^v_mul_f64"), ("dpp", r"_dpp\b|dpp"), ("ldexp", r"^v_ldexp_f64"),
    ("cndmask", r"^v_cndmask"), ("vmov", r"^v_mov_b32(?!.*dpp)|^v_mov_b64"), ("valu_other", r"^v_"),
    ("ds_read", r"^ds_read"), ("ds_write", r"^ds_write"), ("dma", r"^buffer_load.*\blds\b"),
    ("vstore", r"^buffer_store|^global_store"), ("vload", r"^buffer_load|^global_load"),
    ("waitcnt", r"^s_waitcnt"), ("barrier", r"^s_barrier"), ("nop", r"^s_nop"), ("salu", r"^s_"),
]


def classify(op, line):
    for name, rx in CLASSES:
        if name == "dpp":
            if "dpp" in line and op.startswith("v_"):
                return name
            continue
        if re.search(rx, op if name != "dma" else line):
            return name
    return "other"


def main():
    path, kname = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(kname) and ":" in l)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {l.strip()[:-1]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:$", l.strip())}
    for i, l in enumerate(body):
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            c = Counter()
            for x in body[labels[m.group(2)]:i + 1]:
                t = x.strip()
                if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
                    continue
                op = t.split()[0]
                c[classify(op, t)] += 1
            valu = sum(v for k, v in c.items() if k in ("dadd", "dmul", "dpp", "ldexp", "cndmask", "vmov", "valu_other"))
            print(f"loop {m.group(2)} lines {labels[m.group(2)]}-{i}: VALU {valu}  " +
                  " ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
