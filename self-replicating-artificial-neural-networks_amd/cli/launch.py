"""Process launch helpers for the CLIs.

The reference joins an external job pool (``-w/-o/-a`` = port/password/address).  Here a
run is SPMD over ``torch.distributed``: either launched by ``torch.distributed.run`` (env ``RANK`` /
``WORLD_SIZE`` set), or self-launched with ``--nproc N``, which starts ``torch.distributed.run`` as a
*child process* (never an exec) and exits with its status.  The pool flags map to the rendezvous:
``-a`` -> MASTER_ADDR, ``-w`` -> MASTER_PORT; ``-o`` (password) is accepted and ignored.

Recovery: with ``--max-restarts N`` the launcher supervises the run as a child process
(``torch.distributed.run`` for ``--nproc > 1``, the script itself otherwise).  Rank 0 records the
experiment id in ``SERANN_RUN_ID_FILE`` once the run's ``execution_info`` row is saved, and the number
of the last committed generation after each generation; when the child fails -- a crashed rank, or a
rank's generation watchdog (``worker_pool_job_timeout``, utils/faults.py) -- the launcher relaunches it
with ``--resume-experiment-id <id>``, which continues from the last committed generation (exactly,
through the ``resume_state`` table), up to N times.  A relaunch is marked ``SERANN_SUPERVISED_RESUME=1``
(it never extends ``num_generations`` the way a manual resume of a finished run does), and the
supervisor gives up when the watchdog fires twice at the same committed generation: the same work
would only time out again.
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
from typing import List, Optional

RUN_ID_ENV = "SERANN_RUN_ID_FILE"
CHILD_ENV = "SERANN_LAUNCH_CHILD"
RESUME_ENV = "SERANN_SUPERVISED_RESUME"


def add_pool_args(parser):
    parser.add_argument("-w", "--workers-pool-port", required=False, type=int,
                        help="rendezvous port (reference: workers pool server port)")
    parser.add_argument("-o", "--workers-pool-password", required=False,
                        help="accepted for compatibility; torch.distributed needs no password")
    parser.add_argument("-a", "--workers-pool-address", required=False,
                        help="rendezvous address (reference: workers pool server address)")
    parser.add_argument("--nproc", type=int, default=1, help="spawn N local ranks (one per GPU)")
    parser.add_argument("--max-restarts", type=int, default=0,
                        help="relaunch a failed run up to N times, resuming from the last committed generation")


def record_run_id(experiment_id: str, committed_generation: Optional[int] = None) -> None:
    """Rank 0: publish the experiment id (and the last committed generation) for the supervising
    launcher (no-op when unsupervised).  Call it only once the run is resumable: after its
    ``execution_info`` row exists."""
    path = os.environ.get(RUN_ID_ENV)
    if path:
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(str(experiment_id) + ("" if committed_generation is None else f"\n{int(committed_generation)}"))
        os.replace(tmp, path)


def read_run_id(path: str):
    """(experiment id or "", last committed generation or None) from a run-id file."""
    try:
        with open(path) as f:
            parts = f.read().split()
    except FileNotFoundError:
        return "", None
    if not parts:
        return "", None
    return parts[0], (int(parts[1]) if len(parts) > 1 else None)


def _with_resume(argv: List[str], experiment_id: str) -> List[str]:
    """argv with ``--resume-experiment-id <id>`` (any previous -r / --resume-experiment-id replaced)."""
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a in ("-r", "--resume-experiment-id"):
            skip = True
            continue
        if a.startswith("--resume-experiment-id="):
            continue
        out.append(a)
    return out + ["--resume-experiment-id", str(experiment_id)]


def supervise(cmd_for, argv: List[str], max_restarts: int, env: Optional[dict] = None, resume: bool = True) -> int:
    """Run ``cmd_for(argv)`` as a child; on failure relaunch up to ``max_restarts`` times -- with the
    recorded experiment id (``resume``), or unchanged (the evaluation CLI resumes from its output
    pickle by itself).  Returns the last exit status."""
    env = dict(os.environ if env is None else env)
    fd, id_file = tempfile.mkstemp(prefix="serann_run_id_")
    os.close(fd)
    env[RUN_ID_ENV] = id_file
    env[CHILD_ENV] = "1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from ..utils.faults import EXIT_TIMEOUT
    no_timeout = object()                    # sentinel: None is a real value of ``committed`` (nothing committed yet)
    timed_out_at = no_timeout
    try:
        attempt = 0
        while True:
            rc = subprocess.call(cmd_for(argv), env=env)
            if rc == 0 or attempt >= max_restarts:
                return rc
            if not resume:
                attempt += 1
                print(f"[launch] run failed with status {rc}; restart {attempt}/{max_restarts}", file=sys.stderr,
                      flush=True)
                continue
            run_id, committed = read_run_id(id_file)
            if not run_id:
                print(f"[launch] run failed (status {rc}) before the experiment was resumable; not restarting",
                      file=sys.stderr, flush=True)
                return rc
            if rc == EXIT_TIMEOUT:
                if timed_out_at is not no_timeout and timed_out_at == committed:
                    print(f"[launch] the generation watchdog fired again after committed generation {committed}; "
                          f"the same work would time out again: not restarting", file=sys.stderr, flush=True)
                    return rc
                timed_out_at = committed
            attempt += 1
            print(f"[launch] run failed with status {rc}; restart {attempt}/{max_restarts}: resuming experiment "
                  f"{run_id}", file=sys.stderr, flush=True)
            argv = _with_resume(argv, run_id)
            env[RESUME_ENV] = "1"
    finally:
        for f_ in (id_file, id_file + ".tmp"):
            if os.path.exists(f_):
                os.unlink(f_)


def maybe_relaunch(args, script: str, argv: Optional[List[str]] = None, resume: bool = True) -> None:
    """If ``--nproc > 1`` or ``--max-restarts > 0`` and we are not already a launched child / rank,
    run the script as a supervised child process (under torch.distributed.run for several ranks) and
    exit with its return code.  Never an exec: the parent only waits."""
    restarts = int(getattr(args, "max_restarts", 0) or 0)
    if (args.nproc <= 1 and restarts <= 0) or "RANK" in os.environ or os.environ.get(CHILD_ENV):
        if args.workers_pool_address and args.workers_pool_address != "localhost":
            os.environ.setdefault("MASTER_ADDR", args.workers_pool_address)
        if args.workers_pool_port:
            os.environ.setdefault("MASTER_PORT", str(args.workers_pool_port))
        return
    addr = args.workers_pool_address if args.workers_pool_address not in (None, "localhost") else "127.0.0.1"
    port = str(args.workers_pool_port or 29500)
    argv = list(sys.argv[1:] if argv is None else argv)

    def cmd_for(a):
        if args.nproc > 1:
            return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.nproc}",
                    f"--master-addr={addr}", f"--master-port={port}", script, *a]
        return [sys.executable, script, *a]

    sys.exit(supervise(cmd_for, argv, restarts, resume=resume))
