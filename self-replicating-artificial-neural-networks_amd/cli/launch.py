"""Process launch helpers for the CLIs.

The reference joins an external job pool (``-w/-o/-a`` = port/password/address).  Here a
run is SPMD over ``torch.distributed``: either launched by ``torch.distributed.run`` (env ``RANK`` /
``WORLD_SIZE`` set), or self-launched with ``--nproc N``, which starts ``torch.distributed.run`` as a
*child process* (never an exec) and exits with its status.  The pool flags map to the rendezvous:
``-a`` -> MASTER_ADDR, ``-w`` -> MASTER_PORT; ``-o`` (password) is accepted and ignored.

Recovery: with ``--max-restarts N`` the launcher supervises the run as a child process
(``torch.distributed.run`` for ``--nproc > 1``, the script itself otherwise).  Rank 0 records the
experiment id in ``SERANN_RUN_ID_FILE`` as soon as it is known; when the child fails -- a crashed rank,
or a rank's generation watchdog (``worker_pool_job_timeout``, utils/faults.py) -- the launcher relaunches
it with ``--resume-experiment-id <id>``, which continues from the last committed generation (exactly,
through the ``resume_state`` table), up to N times.
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
from typing import List, Optional

RUN_ID_ENV = "SERANN_RUN_ID_FILE"
CHILD_ENV = "SERANN_LAUNCH_CHILD"


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


def record_run_id(experiment_id: str) -> None:
    """Rank 0: publish the experiment id for the supervising launcher (no-op when unsupervised)."""
    path = os.environ.get(RUN_ID_ENV)
    if path:
        with open(path, "w") as f:
            f.write(str(experiment_id))


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
            with open(id_file) as f:
                run_id = f.read().strip()
            if not run_id:
                print(f"[launch] run failed (status {rc}) before an experiment id was recorded; not restarting",
                      file=sys.stderr, flush=True)
                return rc
            attempt += 1
            print(f"[launch] run failed with status {rc}; restart {attempt}/{max_restarts}: resuming experiment "
                  f"{run_id}", file=sys.stderr, flush=True)
            argv = _with_resume(argv, run_id)
    finally:
        os.unlink(id_file)


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
