#!/usr/bin/env python
"""Wall time of the captured training step (graph replay, multi-stream) on a fixed generator-sampled
population: engine.fit() for one epoch of synthetic MNIST-shaped data, timed per step.  Unlike
bench_kernels.py (isolated launches) this measures what a generation actually pays per step."""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=125)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--streams", default="4")
    ap.add_argument("--max-steps", type=int, default=None, help="steps per epoch (profiling runs)")
    ap.add_argument("--ancestor-frac", type=float, default=0.0,
                    help="fraction of the population that are clones of the example.json ancestor (table codec), "
                         "as in the bench's evolved generations")
    ap.add_argument("--population-file", default=None,
                    help="JSON list of source codes (bench.py --dump-population): the bench's evolved population")
    a = ap.parse_args()
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.genome.codec import decoded_form
    from serann.genome.generator import generate
    from serann.genome.interpreter import try_interpret

    df = generate(a.pop * 3, seed=a.seed, validation_genotype_size=100)
    irs = []
    for s in df["code"]:
        r = try_interpret(decoded_form(s))
        if r.ok and r.parameters_count <= 2e6:
            irs.append(r.ir)
        if len(irs) == a.pop:
            break
    if a.population_file:
        import json
        with open(a.population_file) as f:
            irs = [try_interpret(s).ir for s in json.load(f)][:a.pop]
    if a.ancestor_frac > 0:
        from serann.config import default_parameters
        from serann.experiment.runner import build_codec
        params = default_parameters("example")
        codec = build_codec(params, "table", seed=0)
        anc = try_interpret(codec.decode_to_string(np.asarray(params["ancestor_genotype"])[None])[0]).ir
        k = int(round(a.ancestor_frac * a.pop))
        irs = [anc] * k + irs[:a.pop - k]
    data = get_serann_data(synthetic_encodings(), synthetic_mnist())
    for ns in a.streams.split(","):
        os.environ["SERANN_STREAMS"] = ns
        cfg = TrainConfig(epochs=a.epochs, batch_size=750, val_every_epoch=False, max_steps_per_epoch=a.max_steps)
        torch.cuda.synchronize()
        ti = time.perf_counter()
        eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        torch.cuda.synchronize()
        init_s = time.perf_counter() - ti
        t0 = time.perf_counter()
        fit = eng.fit(data, cfg)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"streams={ns} organisms={len(irs)} steps={fit.steps} init_s={init_s:.3f} plan_s={eng.timings['plan_s']:.3f} "
              f"loop_s={fit.learning_time:.3f} ms/step={1e3 * fit.learning_time / fit.steps:.2f} "
              f"launches/step={eng.timings['launches_per_step']} fit_wall={wall:.2f} "
              f"replay_ms/step={eng.timings.get('replay_ms_per_step', float('nan')):.2f}", flush=True)
        eng.close()
        del eng


if __name__ == "__main__":
    main()
