"""Fault injection for recovery tests.

The reference delegates failure handling to its external job pool (per-job timeouts, re-dispatch;
evolutionary_experiment/config.py:7, run_experiment.py:100-108) and has no fault injection.  Here the
recovery point is the per-generation SQLite commit (``generations`` + ``serann`` rows and the additive
``resume_state`` row), and recovery is a relaunch with ``--resume-experiment-id``.  This module lets a
test (or an operator rehearsing a rank loss) kill a rank at a chosen generation:

    SERANN_FAULT_INJECT="generation=2"                 # every rank raises InjectedFault at generation 2
    SERANN_FAULT_INJECT="generation=2,rank=1"          # only rank 1
    SERANN_FAULT_INJECT="generation=2,rank=1,mode=exit"  # rank 1 exits with status 75 (simulated death)

The fault fires at the start of the generation, before any training or DB write of it, so the DB
holds exactly the generations before it.
"""
from __future__ import annotations

import os
from typing import Optional

ENV = "SERANN_FAULT_INJECT"
EXIT_STATUS = 75


class InjectedFault(RuntimeError):
    pass


def parse(spec: Optional[str]) -> Optional[dict]:
    if not spec:
        return None
    out = {"generation": None, "rank": None, "mode": "raise"}
    for item in spec.split(","):
        key, _, val = item.strip().partition("=")
        if key not in out or not val:
            raise ValueError(f"{ENV}: bad item {item!r} (expected generation=G[,rank=R][,mode=raise|exit])")
        out[key] = val if key == "mode" else int(val)
    if out["generation"] is None:
        raise ValueError(f"{ENV}: generation=G is required")
    if out["mode"] not in ("raise", "exit"):
        raise ValueError(f"{ENV}: mode must be raise or exit")
    return out


def maybe_inject(generation: int, rank: int = 0, spec: Optional[str] = None) -> None:
    f = parse(os.environ.get(ENV) if spec is None else spec)
    if f is None or f["generation"] != int(generation) or (f["rank"] is not None and f["rank"] != int(rank)):
        return
    if f["mode"] == "exit":
        os._exit(EXIT_STATUS)
    raise InjectedFault(f"injected fault: rank {rank} at generation {generation}")
