"""roctx ranges (visible in ``rocprofv3 --marker-trace`` / kernel traces) + a cheap host timer.

On ROCm, ``torch.cuda.nvtx`` is backed by roctx (libroctx64 ships with torch), so
ranges around prefill / decode / collectives show up by name next to the K1-K6
kernels. Disabled (zero-cost) unless ``ROUNDTABLE_TRACE=1``.
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Dict, Iterator

_ENABLED = os.environ.get("ROUNDTABLE_TRACE") == "1"
TIMERS: Dict[str, float] = {}


@contextlib.contextmanager
def range(name: str) -> Iterator[None]:  # noqa: A001 - mirrors nvtx.range
    if not _ENABLED:
        yield
        return
    import torch
    pushed = False
    try:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:  # noqa: BLE001 - tracing must never break inference
        pushed = False
    t0 = time.perf_counter()
    try:
        yield
    finally:
        TIMERS[name] = TIMERS.get(name, 0.0) + time.perf_counter() - t0
        if pushed:
            torch.cuda.nvtx.range_pop()
