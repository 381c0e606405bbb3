#!/usr/bin/env python
"""BASELINE config #5 on one GPU: retrospective evaluation of sampled genotypes (serann_evaluation).

Each genotype: E = num_evaluations identical replicas trained jointly for 5 epochs (batch 750), R =
replications_per_evaluation offspring per replica, proofreading, decode, validity and mutation-rate
histograms (reference serann_evaluation/logic.py:153-231, parameters/general.json: E = 50, R = 100).
Several genotypes share one homogeneous population engine (``evaluate_many``).  Reports seconds per
evaluated genotype; the reference gives each genotype a job timeout of 800 s
(serann_evaluation/run_evaluation.py:184) and publishes no measured time.  Synthetic data and the table
codec (no network, no trained RiboAE)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genotypes", type=int, default=4)
    ap.add_argument("--per-engine", type=int, default=2)
    ap.add_argument("--evaluations", type=int, default=50)
    ap.add_argument("--replications", type=int, default=100)
    ap.add_argument("--max-steps", type=int, default=None, help="CPU smoke runs only (never for timing)")
    a = ap.parse_args()
    from serann.config import default_parameters
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.evaluation.evaluator import SerannEvaluator
    from serann.experiment.runner import build_codec

    params = default_parameters("example")
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    codec = build_codec(params, "table", seed=0)
    data = get_serann_data(synthetic_encodings(), synthetic_mnist())
    from serann.engine.base import TrainConfig
    cfg = TrainConfig(epochs=int(params["training_epochs"]), batch_size=int(params["training_batch_size"]),
                      max_steps_per_epoch=a.max_steps)
    ev = SerannEvaluator(params, data, codec, train_cfg=cfg, num_evaluations=a.evaluations, replications_per_evaluation=a.replications,
                         engine="hip" if dev == "cuda" else "torch", device=dev,
                         max_parameters=float(params["max_serann_parameters"]))
    rng = np.random.default_rng(0)
    pool = []
    while len(pool) < a.genotypes + a.per_engine:           # valid, trainable genotypes of the codec
        g = rng.integers(0, 2, int(params["genotype_size"]))
        src = codec.decode_to_string(g[None])[0]
        r = ev.cache(src)
        if r.ok and r.parameters_count <= float(params["max_serann_parameters"]):
            pool.append(g)
    ev.evaluate_many(pool[:a.per_engine])                    # warm-up (plan compile, first touch)
    if dev == "cuda":
        torch.cuda.synchronize()
    todo = pool[a.per_engine:]
    ev.timings = {k: 0.0 for k in ev.timings}
    t0 = time.perf_counter()
    res = []
    for i in range(0, len(todo), a.per_engine):
        res += ev.evaluate_many(todo[i:i + a.per_engine])
    if dev == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    acc = [float(np.mean(r["classification_accuracy"])) for r in res if isinstance(r["classification_accuracy"], list)]
    print(json.dumps({"metric": "evaluation_seconds_per_genotype", "value": dt / len(todo), "unit": "s",
                      "genotypes": len(todo), "replicas_per_genotype": a.evaluations,
                      "offspring_per_replica": a.replications, "genotypes_per_engine": a.per_engine,
                      "reference_job_timeout_s": 800, "mean_val_acc": float(np.mean(acc)) if acc else None,
                      "phase_seconds_per_genotype": {k: v / len(todo) for k, v in ev.timings.items()},
                      "device": dev, "data": "synthetic, table codec"}))


if __name__ == "__main__":
    main()
