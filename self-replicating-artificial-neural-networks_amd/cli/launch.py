"""Process launch helpers for the CLIs.

The reference joins an external job pool (``-w/-o/-a`` = port/password/address).  Here a
run is SPMD over ``torch.distributed``: either launched by ``torch.distributed.run`` (env ``RANK`` /
``WORLD_SIZE`` set), or self-launched with ``--nproc N``, which starts ``torch.distributed.run`` as a
*child process* (never an exec) and exits with its status.  The pool flags map to the rendezvous:
``-a`` -> MASTER_ADDR, ``-w`` -> MASTER_PORT; ``-o`` (password) is accepted and ignored.
"""
from __future__ import annotations

import os
import subprocess
import sys


def add_pool_args(parser):
    parser.add_argument("-w", "--workers-pool-port", required=False, type=int,
                        help="rendezvous port (reference: workers pool server port)")
    parser.add_argument("-o", "--workers-pool-password", required=False,
                        help="accepted for compatibility; torch.distributed needs no password")
    parser.add_argument("-a", "--workers-pool-address", required=False,
                        help="rendezvous address (reference: workers pool server address)")
    parser.add_argument("--nproc", type=int, default=1, help="spawn N local ranks (one per GPU)")


def maybe_relaunch(args, script: str) -> None:
    """If ``--nproc > 1`` and we are not already a distributed rank, run the script under
    torch.distributed.run as a child process and exit with its return code."""
    if args.nproc <= 1 or "RANK" in os.environ:
        if args.workers_pool_address and args.workers_pool_address != "localhost":
            os.environ.setdefault("MASTER_ADDR", args.workers_pool_address)
        if args.workers_pool_port:
            os.environ.setdefault("MASTER_PORT", str(args.workers_pool_port))
        return
    addr = args.workers_pool_address if args.workers_pool_address not in (None, "localhost") else "127.0.0.1"
    port = str(args.workers_pool_port or 29500)
    argv = [a for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.nproc}",
           f"--master-addr={addr}", f"--master-port={port}", script, *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = subprocess.call(cmd, env=env)
    sys.exit(rc)
