"""Phase tracing.

The reference only times ``fit`` and ``predict`` (experiment_worker.py:114-119, 135, 165) and the whole
generation (experiment.py:101-108).  ``phase(name)`` brackets a generation phase so it shows up in:

* ``torch.profiler`` traces (``record_function``; free when no profiler is active);
* rocprofv3 marker traces (``--marker-trace``): with ``SERANN_ROCTX=1`` every phase is also a
  roctx range (``torch.cuda.nvtx`` is roctx on ROCm builds);
* a per-phase wall-clock accumulator (``PhaseTimer``) that the generation loop writes to its JSONL
  perf log.

``profiled(dir)`` wraps a region in ``torch.profiler.profile`` (CPU + HIP activities) and exports a
Chrome trace per call, for ``bench.py --profile-dir``-style one-off captures.
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Dict, Optional

_ROCTX = os.environ.get("SERANN_ROCTX", "0") == "1"


def _roctx():
    if not _ROCTX:
        return None
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:                                   # pragma: no cover - torch always importable here
        pass
    return None


class PhaseTimer:
    """Accumulates wall seconds per phase name."""

    def __init__(self):
        self.seconds: Dict[str, float] = {}

    def add(self, name: str, dt: float) -> None:
        self.seconds[name] = self.seconds.get(name, 0.0) + dt

    def reset(self) -> Dict[str, float]:
        out, self.seconds = self.seconds, {}
        return out


@contextlib.contextmanager
def phase(name: str, timer: Optional[PhaseTimer] = None):
    import torch
    nv = _roctx()
    if nv is not None:
        nv.range_push(name)
    t0 = time.perf_counter()
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if timer is not None:
            timer.add(name, time.perf_counter() - t0)
        if nv is not None:
            nv.range_pop()


@contextlib.contextmanager
def profiled(out_dir: Optional[str], tag: str = "trace"):
    """torch.profiler capture of the enclosed region into ``out_dir/<tag>.json`` (no-op if None)."""
    if not out_dir:
        yield None
        return
    import torch
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)              # HIP activities on ROCm
    os.makedirs(out_dir, exist_ok=True)
    with profile(activities=acts, record_shapes=False) as prof:
        yield prof
    prof.export_chrome_trace(os.path.join(out_dir, f"{tag}.json"))
