#!/usr/bin/env python
"""Phase timing of one shard worker generation (engine construction, plan compile, training loop,
test evaluation, replication) on a fixed population -- what a generation pays outside the step loop."""
from __future__ import annotations

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    from serann.config import default_parameters
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig, replication_image_rows
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.experiment.runner import build_codec
    from serann.genome.codec import decoded_form
    from serann.genome.generator import generate
    from serann.genome.interpreter import try_interpret

    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("frac", nargs="?", type=float, default=0.8)
    ap.add_argument("--population-file", default=None,
                    help="JSON list of source codes (bench.py --dump-population): the bench's evolved population")
    a = ap.parse_args()
    pop, frac = 125, a.frac
    df = generate(pop * 3, seed=11, validation_genotype_size=100)
    irs = [r.ir for r in (try_interpret(decoded_form(s)) for s in df["code"]) if r.ok and r.parameters_count <= 2e6][:pop]
    params = default_parameters("example")
    codec = build_codec(params, "table", seed=0)
    anc = try_interpret(codec.decode_to_string(np.asarray(params["ancestor_genotype"])[None])[0]).ir
    k = int(round(frac * pop))
    irs = [anc] * k + irs[:pop - k]
    if a.population_file:
        import json
        with open(a.population_file) as f:
            irs = [try_interpret(s).ir for s in json.load(f)][:pop]
        pop = len(irs)
    data = get_serann_data(synthetic_encodings(), synthetic_mnist())
    cfg = TrainConfig(epochs=5, batch_size=750)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        fit = eng.fit(data, cfg)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        acc = eng.evaluate(data.test_x, data.test_labels, data.test_g, cfg)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        R = 50
        imgs = [data.test_x[replication_image_rows(q, R, pop * R, len(data.test_x))] for q in range(pop)]
        eng.replicate(np.asarray(data.test_g[:pop], np.float32), imgs, cfg)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        eng.close()
        print(f"rep {rep}: init {t1 - t0:.3f}s  fit {t2 - t1:.3f}s (plan {eng.timings['plan_s']:.3f}s, loop "
              f"{fit.learning_time:.3f}s, {fit.steps} steps)  test-eval {t3 - t2:.3f}s  replicate {t4 - t3:.3f}s",
              flush=True)


if __name__ == "__main__":
    main()
