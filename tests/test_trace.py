"""Phase tracing and torch.profiler capture on the CPU."""
import json
import os

import torch

from serann.utils.trace import PhaseTimer, phase, profiled


def test_phase_timer_and_profiler_ranges(tmp_path):
    timer = PhaseTimer()
    with profiled(str(tmp_path), "t"):
        with phase("outer", timer):
            with phase("inner", timer):
                torch.ones(64, 64) @ torch.ones(64, 64)
        with phase("inner", timer):
            pass
    secs = timer.reset()
    assert set(secs) == {"outer", "inner"} and secs["outer"] >= 0 and timer.seconds == {}
    trace = json.load(open(os.path.join(tmp_path, "t.json")))
    names = {e.get("name") for e in trace["traceEvents"]}
    assert {"outer", "inner"} <= names


def test_profiled_none_is_noop():
    with profiled(None) as p:
        assert p is None
