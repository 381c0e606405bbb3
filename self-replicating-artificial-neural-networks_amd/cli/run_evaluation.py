"""``run_evaluation`` CLI (reference: serann_evaluation/run_evaluation.py:135-197).

    python serann_evaluation/run_evaluation.py -p serann_evaluation/parameters/general.json -n NAME
        [-c cached.csv] [-s] [-w PORT -a ADDR] [--nproc N] [--engine ...] [--batch K]

Loads the experiment results (``serann`` or legacy ``srann`` table), samples with the configured
sampler, evaluates over all ranks and writes ``data/serann_evaluations/<NAME>.pkl``.  Parameter
files without ``experiment_params`` (3 of the reference's 4) fall back to the
values stored in the experiment's ``execution_info``.
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path

import numpy as np
import pandas as pd

EXPERIMENT_PARAM_KEYS = ["max_tokens", "genotype_size", "error_correction_probability",
                         "classification_image_dimensions", "num_classification_classes", "training_epochs",
                         "training_batch_size"]


def get_args(argv=None):
    p = argparse.ArgumentParser(description="Retrospective SeRANN evaluation")
    p.add_argument("-p", "--parameters", required=True, help="Parameters file path")
    p.add_argument("-n", "--output-name", required=True, help="Evaluation file name")
    p.add_argument("-c", "--cached-evaluations", required=False, help="Use evaluations from this file as cache")
    p.add_argument("-s", "--no-shared-cache", default=False, action="store_true",
                   help="Don't share cache between workers")
    from .launch import add_pool_args
    add_pool_args(p)
    p.add_argument("--engine", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("--codec", default="auto", choices=["auto", "riboae", "table"])
    p.add_argument("--batch", type=int, default=4, help="genotypes evaluated together in one engine per rank")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--data-subset", type=int, default=None)
    p.add_argument("--strict-reference", action="store_true")
    return p.parse_args(argv)


def update_workers_with_cached_evaluations(evaluations_path, df, worker):
    """Seed the genotype cache from a CSV of earlier evaluations (run_evaluation.py:114-132)."""
    sample = pd.read_csv(evaluations_path)
    visited = sample[sample["visited"] == True]  # noqa: E712
    ids = df.index.intersection(visited["serann_id"].drop_duplicates().values)
    keys = df.loc[ids, "genotype_hex"]
    cache = {}
    for sid, grp in visited.set_index("serann_id").loc[ids].groupby(level=0):
        g = grp.drop_duplicates(subset=["proofreading_strength"]) if "proofreading_strength" in grp else grp
        rec = {"classification_accuracy": float(g["classification_accuracy"].mean())}
        if "proofreading_strength" in g:
            rec["mutation_rate"] = {r["proofreading_strength"]: r["mutation_rate"] for _, r in g.iterrows()}
            rec["offspring_viability"] = {r["proofreading_strength"]: r["offspring_viability"] for _, r in g.iterrows()}
        cache[keys.loc[sid]] = rec
    worker.handle_update(cache)


def main(argv=None, script=None):
    args = get_args(argv)
    from .launch import maybe_relaunch
    from pathlib import Path
    maybe_relaunch(args, script or str(Path(__file__).resolve().parents[2] / "serann_evaluation" / "run_evaluation.py"),
                   argv, resume=False)

    from ..analysis.results import load_experiment_results
    from ..config import experiment_config as config
    from ..evaluation.driver import SAMPLERS, SampleDeepEvaluator
    from ..evaluation.evaluator import SerannEvaluationWorker
    from ..experiment.runner import build_codec, default_device, default_engine
    from ..data.datasets import get_serann_data, load_encodings, load_mnist
    from ..parallel.comm import make_comm
    from ..utils.db import ExperimentDB

    comm = make_comm()
    with open(args.parameters) as f:
        parameters = json.load(f)
    df = None
    if comm.is_root:
        print("Loading data", flush=True)
        df = load_experiment_results(parameters["experiment_id"])
    df = comm.broadcast_object(df)
    exp_params = parameters.get("experiment_params")
    if exp_params is None:
        db = ExperimentDB(Path(config["experiment_results_dir"]) / f"{parameters['experiment_id']}.sqlite")
        info = comm.broadcast_object(db.get_last_execution_info() if comm.is_root else None)
        exp_params = {k: info[k] for k in EXPERIMENT_PARAM_KEYS if k in info}
        exp_params.setdefault("max_tokens", 350)
    print_ = print if comm.is_root else (lambda *a, **k: None)
    print_("Sampling examples to evaluate", flush=True)
    if parameters["sampler"] not in SAMPLERS:
        raise SystemExit("Unknown sampler")
    sample = SAMPLERS[parameters["sampler"]](seed=args.seed).sample(df, parameters).drop_duplicates()

    device = default_device(comm)
    engine = default_engine(device) if args.engine == "auto" else args.engine
    encodings = load_encodings(genotype_size=int(exp_params["genotype_size"]))
    data = get_serann_data(encodings, load_mnist(), int(exp_params["num_classification_classes"]),
                           n_train=args.data_subset)
    codec = build_codec(exp_params, args.codec, device=device)
    worker = SerannEvaluationWorker(exp_params, data, codec, parameters["num_evaluations"],
                                    parameters["replications_per_evaluation"], engine=engine, device=device,
                                    seed=args.seed, strict_reference=args.strict_reference)
    if args.cached_evaluations is not None:
        update_workers_with_cached_evaluations(args.cached_evaluations, df, worker)
    output_path = Path(config["serann_evaluations_dir"]) / (args.output_name + ".pkl")
    if comm.is_root:
        output_path.parent.mkdir(exist_ok=True, parents=True)
    ev = SampleDeepEvaluator(df, str(output_path), sample, worker, comm=comm,
                             shared_cache=not args.no_shared_cache, batch=args.batch)
    ev.run()
    comm.shutdown()
    return str(output_path)


if __name__ == "__main__":
    main()
