"""``run_experiment`` CLI (reference: evolutionary_experiment/run_experiment.py:19-114).

Same flags (``-p -r -s -w -o -a``) plus ``--engine {auto,hip,torch}``, ``--codec {auto,riboae,table}``,
``--nproc``, ``--max-generations``, ``--perf-log``, ``--data-subset`` (CPU smoke runs only).
Creates ``data/experiment_results/<uuid>.sqlite`` (or resumes one), records host / dataset / codec /
seed in ``execution_info`` and runs the generation loop over all ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import uuid
from pathlib import Path

import numpy as np


def get_args(argv=None):
    p = argparse.ArgumentParser(description="Run a SeRANN evolutionary experiment")
    p.add_argument("-p", "--parameters", required=False, help="Experiment parameters file path")
    p.add_argument("-r", "--resume-experiment-id", required=False, help="Experiment ID to resume")
    p.add_argument("-s", "--random-seed", required=False, help="Override random seed")
    from .launch import add_pool_args
    add_pool_args(p)
    p.add_argument("--engine", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("--codec", default="auto", choices=["auto", "riboae", "table"])
    p.add_argument("--max-generations", type=int, default=None)
    p.add_argument("--perf-log", default=None)
    p.add_argument("--data-subset", type=int, default=None, help="use only the first N training images (smoke)")
    p.add_argument("--strict-reference", action="store_true",
                   help="reproduce the reference's crash when a parent has more offspring than its pool")
    return p.parse_args(argv)


def main(argv=None, script=None):
    args = get_args(argv)
    from .launch import RESUME_ENV, maybe_relaunch, record_run_id
    maybe_relaunch(args, script or str(Path(__file__).resolve().parents[2] / "evolutionary_experiment" /
                                       "run_experiment.py"), argv)

    from ..config import experiment_config as config
    from ..experiment.experiment import Experiment
    from ..experiment.runner import setup
    from ..parallel.comm import make_comm
    from ..utils.db import ExperimentDB

    comm = make_comm()
    results_dir = Path(config["experiment_results_dir"])
    if comm.is_root:
        results_dir.mkdir(exist_ok=True, parents=True)

    start_generation = 0
    stored_seed = None
    if args.resume_experiment_id is None:
        if not args.parameters:
            raise SystemExit("--parameters is required for a new experiment")
        experiment_id = comm.broadcast_object(str(uuid.uuid4()) if comm.is_root else None)
        with open(args.parameters) as f:
            parameters = json.load(f)
        db = ExperimentDB(results_dir / f"{experiment_id}.sqlite") if comm.is_root else None
    else:
        experiment_id = args.resume_experiment_id
        db = ExperimentDB(results_dir / f"{experiment_id}.sqlite") if comm.is_root else None
        state = None
        if comm.is_root:
            start_generation = db.get_generations_count()
            info = db.get_last_execution_info()
            # the per-organism weight-init and epoch-permutation seeds derive from random_seed: a resume
            # without -s continues with the seed the run was started with
            if "random_seed" in info and info["random_seed"] is not None and str(info["random_seed"]) != "nan":
                stored_seed = int(info["random_seed"])
            if args.parameters is not None:
                with open(args.parameters) as f:
                    parameters = json.load(f)
            else:
                parameters = {k: v for k, v in info.drop("start_time").items()}
                for k in ("host_name", "encodings_dataset", "tokens_vocabulary", "ribosomal_autoencoder", "random_seed"):
                    parameters.pop(k, None)
                # a manual resume of a finished run extends it (reference run_experiment.py:93-95); a
                # supervised relaunch after the last generation must not run a second set
                if start_generation == parameters["num_generations"] and not os.environ.get(RESUME_ENV):
                    parameters["num_generations"] *= 2
            state = (start_generation, parameters, stored_seed)
        start_generation, parameters, stored_seed = comm.broadcast_object(state)

    if args.random_seed is not None:
        seed = int(args.random_seed)
    elif stored_seed is not None:
        seed = stored_seed
    else:
        seed = int(config["random_seed"])
    np.random.seed(seed)

    s = setup(parameters, engine=args.engine, codec=args.codec, comm=comm, n_train=args.data_subset)
    parameters["host_name"] = socket.gethostname()
    parameters["encodings_dataset"] = Path(config["encodings_dataset_path"]).stem
    parameters["tokens_vocabulary"] = Path(config["vocabulary_path"]).stem
    parameters["ribosomal_autoencoder"] = s.codec.get_model_name()
    parameters["random_seed"] = seed
    if comm.is_root:
        print(f"Experiment id: {experiment_id} | ranks: {comm.world_size} | engine: {s.engine} | "
              f"codec: {s.codec.get_model_name()} | data: {'synthetic' if s.data.synthetic else 'MNIST'}", flush=True)
    exp = Experiment(experiment_id, s.encodings, s.worker, db, parameters, s.codec, comm=comm,
                     start_generation=start_generation, random_seed=seed, strict_reference=args.strict_reference,
                     perf_log=args.perf_log)
    if comm.is_root:
        # resumable from here on (execution_info is saved): tell a supervising launcher, then keep it told
        # which generation was committed last
        record_run_id(experiment_id, start_generation - 1 if start_generation > 0 else None)
    exp.execute(max_generations=args.max_generations,
                on_generation=(lambda g, rec: record_run_id(experiment_id, g)) if comm.is_root else None)
    comm.shutdown()
    return experiment_id


if __name__ == "__main__":
    main()
