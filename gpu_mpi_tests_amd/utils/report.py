"""Machine-readable result records (one JSON object per line).

The native apps write the same records with ``--json=FILE``
(csrc/include/gmt/util.hpp ``JsonRecord``); scripts/bench_sweep.py merges both.
"""
from __future__ import annotations

import json
import math


def _clean(v):
    if isinstance(v, float) and not math.isfinite(v):
        return None
    if isinstance(v, dict):
        return {k: _clean(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_clean(x) for x in v]
    return v


def json_line(rec: dict) -> str:
    return json.dumps(_clean(rec), sort_keys=False)


def write_jsonl(path: str | None, rec: dict) -> None:
    if not path:
        return
    with open(path, "a") as f:
        f.write(json_line(rec) + "\n")
