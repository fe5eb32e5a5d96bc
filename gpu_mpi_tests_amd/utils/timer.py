"""Wall-clock / device timers and robust statistics (min / median / mean).

Reference timers: MPI_Wtime and clock_gettime(CLOCK_MONOTONIC) around single
calls (mpi_daxpy_nvtx.cc:242-291; mpi_stencil2d_gt.cc:512-526).  Here every
measurement is a sample in ``Stats`` so reports carry the distribution, and
``Timer`` synchronises the device on both sides when it is a GPU.
"""
from __future__ import annotations

import statistics
import time
from dataclasses import dataclass, field

import torch


@dataclass
class Stats:
    samples: list = field(default_factory=list)

    def add(self, v: float) -> None:
        self.samples.append(float(v))

    @property
    def n(self) -> int:
        return len(self.samples)

    def total(self) -> float:
        return sum(self.samples)

    def mean(self) -> float:
        return statistics.fmean(self.samples) if self.samples else 0.0

    def median(self) -> float:
        return statistics.median(self.samples) if self.samples else 0.0

    def min(self) -> float:
        return min(self.samples) if self.samples else 0.0

    def max(self) -> float:
        return max(self.samples) if self.samples else 0.0

    def summary(self) -> dict:
        return {"n": self.n, "min": self.min(), "median": self.median(), "mean": self.mean(),
                "max": self.max()}


class Timer:
    """``with Timer(device) as t: ...`` then ``t.elapsed`` (seconds)."""

    def __init__(self, device: torch.device | str | None = None, stats: Stats | None = None):
        self.device = torch.device(device) if device is not None else None
        self.stats = stats
        self.elapsed = 0.0

    def _sync(self):
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def __enter__(self):
        self._sync()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self._sync()
        self.elapsed = time.perf_counter() - self.t0
        if self.stats is not None:
            self.stats.add(self.elapsed)
        return False
