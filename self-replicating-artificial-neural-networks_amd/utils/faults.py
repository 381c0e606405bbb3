"""Fault injection for recovery tests, and the per-generation watchdog.

The reference delegates failure handling to its external job pool (per-job timeouts, re-dispatch;
evolutionary_experiment/config.py:7, run_experiment.py:100-108) and has no fault injection.  Here the
recovery point is the per-generation SQLite commit (``generations`` + ``serann`` rows and the additive
``resume_state`` row), and recovery is a relaunch with ``--resume-experiment-id``.  This module lets a
test (or an operator rehearsing a rank loss) kill a rank at a chosen generation:

    SERANN_FAULT_INJECT="generation=2"                 # every rank raises InjectedFault at generation 2
    SERANN_FAULT_INJECT="generation=2,rank=1"          # only rank 1
    SERANN_FAULT_INJECT="generation=2,rank=1,mode=exit"  # rank 1 exits with status 75 (simulated death)

    SERANN_FAULT_INJECT="generation=2,mode=hang"       # every rank stalls (the watchdog must fire)
    SERANN_FAULT_INJECT="evaluated=100,mode=exit"      # run_evaluation dies after its first saved 100 results

The fault fires at the start of the generation, before any training or DB write of it, so the DB
holds exactly the generations before it.

:class:`GenerationWatchdog` replaces the job pool's per-job timeout (``worker_pool_job_timeout = 1080`` s,
evolutionary_experiment/config.py:7): a rank whose generation work exceeds it prints the stall and exits
with status ``EXIT_TIMEOUT`` -- under ``torch.distributed.run`` the other ranks are torn down, and the
launcher (``cli/launch.py --max-restarts``) relaunches the run with ``--resume-experiment-id``, which
resumes from the last committed generation.
"""
from __future__ import annotations

import os
from typing import Optional

import sys
import threading
import time

ENV = "SERANN_FAULT_INJECT"
EXIT_STATUS = 75
EXIT_TIMEOUT = 76


class InjectedFault(RuntimeError):
    pass


def parse(spec: Optional[str]) -> Optional[dict]:
    if not spec:
        return None
    out = {"generation": None, "evaluated": None, "rank": None, "mode": "raise"}
    for item in spec.split(","):
        key, _, val = item.strip().partition("=")
        if key not in out or not val:
            raise ValueError(f"{ENV}: bad item {item!r} (expected generation=G|evaluated=N[,rank=R]"
                             f"[,mode=raise|exit|hang])")
        out[key] = val if key == "mode" else int(val)
    if (out["generation"] is None) == (out["evaluated"] is None):
        raise ValueError(f"{ENV}: exactly one of generation=G, evaluated=N is required")
    if out["mode"] not in ("raise", "exit", "hang"):
        raise ValueError(f"{ENV}: mode must be raise, exit or hang")
    return out


def maybe_inject(generation: int, rank: int = 0, spec: Optional[str] = None) -> None:
    f = parse(os.environ.get(ENV) if spec is None else spec)
    if f is None or f["generation"] is None or f["generation"] != int(generation) or \
            (f["rank"] is not None and f["rank"] != int(rank)):
        return
    _fire(f, f"rank {rank} at generation {generation}")


def maybe_inject_evaluation(saved: int, rank: int = 0, spec: Optional[str] = None) -> None:
    """Evaluation recovery tests: fire once ``saved`` results (already pickled) reach ``evaluated=N``."""
    f = parse(os.environ.get(ENV) if spec is None else spec)
    if f is None or f["evaluated"] is None or int(saved) < f["evaluated"] or \
            (f["rank"] is not None and f["rank"] != int(rank)):
        return
    _fire(f, f"rank {rank} after {saved} saved evaluations")


def _fire(f: dict, what: str) -> None:
    if f["mode"] == "exit":
        os._exit(EXIT_STATUS)
    if f["mode"] == "hang":
        while True:                    # a stalled rank: only the watchdog ends this
            time.sleep(1.0)
    raise InjectedFault(f"injected fault: {what}")


JOB_ORGANISMS = 112      # organisms per pool job in the reference split (logic/experiment.py:170-178)


def job_scale(n_organisms: int, waves: int = 1) -> float:
    """How many reference pool jobs a shard of ``n_organisms`` (trained in ``waves`` sequential waves) is."""
    return float(max(1, -(-int(n_organisms) // JOB_ORGANISMS), int(waves)))


class GenerationWatchdog:
    """Arms a timer for the work of one generation; if it is not disarmed within ``timeout_s`` the
    process reports the stall on stderr and exits with ``EXIT_TIMEOUT`` (``os._exit``: a stalled device
    call or collective cannot be interrupted from Python).  ``timeout_s <= 0`` disables it."""

    def __init__(self, timeout_s: float, rank: int = 0, exit_status: int = EXIT_TIMEOUT):
        self.timeout_s = float(timeout_s)
        self.rank = int(rank)
        self.exit_status = int(exit_status)
        self._timer: Optional[threading.Timer] = None
        self._label = ""
        self._armed_s = self.timeout_s

    def _fire(self):
        sys.stderr.write(f"[watchdog] rank {self.rank}: {self._label} exceeded its timeout of "
                         f"{self._armed_s:.0f} s (worker_pool_job_timeout per job); exiting with status "
                         f"{self.exit_status} for a relaunch with --resume-experiment-id\n")
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(self.exit_status)

    def arm(self, label: str = "generation", scale: float = 1.0) -> "GenerationWatchdog":
        """(Re-)arm for ``scale`` x ``timeout_s``: the reference's timeout bounded one pool job of at most
        ``JOB_ORGANISMS`` organisms, so a rank's shard of n organisms gets ceil(n / JOB_ORGANISMS) jobs'
        worth (:func:`job_scale`)."""
        self.disarm()
        self._label = label
        self._armed_s = self.timeout_s * max(1.0, float(scale))
        if self.timeout_s > 0:
            self._timer = threading.Timer(self._armed_s, self._fire)
            self._timer.daemon = True
            self._timer.start()
        return self

    def disarm(self):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.disarm()
        return False
