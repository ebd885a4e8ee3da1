"""Tracing / profiling helpers (absent in the reference — SURVEY §5.1).

* ``trace_range(name)``  roctx range (torch.cuda.nvtx maps to roctx on ROCm) so rocprofv3
  ``--marker-trace`` / Perfetto timelines show stages, layers and comm ops; enabled with
  ``EDGELLM_TRACE=1`` (zero cost otherwise).
* ``LatencyHistogram``   per-token latency distribution (p50 / p90 / p99) from device events or
  host timestamps.
* ``MetricsWriter``      structured JSONL records (tok/s, TTFT, latency percentiles, HBM peak).
* ``debug_sync()``       ``EDGELLM_SYNC_DEBUG=1`` forces a device synchronise after an op so a
  faulting kernel is reported at its call site (the race-detection debug mode of SURVEY §5.2;
  use with ``AMD_SERIALIZE_KERNEL=3`` / ``HIP_LAUNCH_BLOCKING=1``).
"""
from __future__ import annotations

import contextlib
import json
import os
import time
from typing import Dict, Iterable, List, Optional

import torch

TRACE = os.environ.get("EDGELLM_TRACE", "0") == "1"
SYNC_DEBUG = os.environ.get("EDGELLM_SYNC_DEBUG", "0") == "1"


@contextlib.contextmanager
def trace_range(name: str):
    if TRACE and torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


def debug_sync(where: str = ""):
    if SYNC_DEBUG and torch.cuda.is_available():
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError(f"device fault detected after {where}: {e}") from e


class LatencyHistogram:
    def __init__(self):
        self.samples: List[float] = []

    def add(self, ms: float):
        self.samples.append(float(ms))

    def extend(self, vals: Iterable[float]):
        self.samples.extend(float(v) for v in vals)

    def percentile(self, p: float) -> float:
        if not self.samples:
            return float("nan")
        s = sorted(self.samples)
        k = min(len(s) - 1, max(0, int(round(p / 100.0 * (len(s) - 1)))))
        return s[k]

    def summary(self) -> Dict[str, float]:
        return {"count": len(self.samples), "p50_ms": self.percentile(50), "p90_ms": self.percentile(90),
                "p99_ms": self.percentile(99),
                "mean_ms": sum(self.samples) / len(self.samples) if self.samples else float("nan")}


class MetricsWriter:
    def __init__(self, path: Optional[str]):
        self.path = path

    def write(self, **rec):
        if not self.path:
            return
        rec.setdefault("ts", time.time())
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            rec.setdefault("hbm_peak_gb", torch.cuda.max_memory_allocated() / 1e9)
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")
