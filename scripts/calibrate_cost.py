#!/usr/bin/env python
"""Fit the LPT cost model (serann/experiment/cost_model.py) to measured training-step times, and report
the predicted and measured rank imbalance of the LPT partition.

1. Draw random sub-populations (32..160 organisms, around a pop-1000 / 8-rank shard) of a population (``--population-file``: JSON sources
   from ``bench.py --dump-population``, else a generator sample); train each for a few graph-replayed
   steps on the HIP engine and record the device time per step (engine.timings['replay_ms_per_step']).
2. Fit t = sum_k coef_k * sum(feature_k) + d (cost_model.features: conv / dense FLOPs, BN / other
   activation elements, nodes) by non-negative least squares; print the fit
   and write the coefficients (``--out``, default the package's parameters/cost_model.json).
3. Partition the whole population for 2 / 4 / 8 ranks (LPT on the fitted model) and print predicted
   max/mean rank time; with ``--measure-ranks R`` time each of the R shards on this GPU in turn.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def load_population(a):
    from serann.genome.codec import decoded_form
    from serann.genome.generator import generate
    from serann.genome.interpreter import try_interpret
    if a.population_file:
        with open(a.population_file) as f:
            srcs = json.load(f)
        irs = [r.ir for r in (try_interpret(s) for s in srcs) if r.ok and r.parameters_count <= 2e6]
    else:
        df = generate(a.pop * 3, seed=a.seed, validation_genotype_size=100)
        irs = []
        for s in df["code"]:
            r = try_interpret(decoded_form(s))
            if r.ok and r.parameters_count <= 2e6:
                irs.append(r.ir)
    return irs[:a.pop]


def step_ms(irs, data, steps):
    import torch
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    cfg = TrainConfig(epochs=1, batch_size=750, max_steps_per_epoch=steps, val_every_epoch=False)
    eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
    eng.fit(data, cfg)
    ms = eng.timings["replay_ms_per_step"]
    eng.close()
    del eng
    torch.cuda.empty_cache()
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--population-file", default=None)
    ap.add_argument("--pop", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--subsets", type=int, default=48)
    ap.add_argument("--min-size", type=int, default=32, help="sub-population sizes span the shard sizes LPT forms")
    ap.add_argument("--max-size", type=int, default=160)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--measure-ranks", type=int, default=0)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.experiment import cost_model as CM
    from serann.parallel.partition import lpt_partition
    irs = load_population(a)
    print(f"population: {len(irs)} trainable organisms", flush=True)
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=16000, n_test=1000, seed=1),
                           n_train=16000, n_test=1000)
    names = ["Fc", "Fd", "Ab", "Aa", "N"]

    def row(ir):
        f = CM.features(ir)
        return [f[k] * (3.0 * 750 if k.startswith("F") else 750.0) if k in CM.PER_SAMPLE else f[k] for k in names]
    feats = np.array([row(ir) for ir in irs])
    rng = np.random.default_rng(a.seed)
    X, y = [], []
    t0 = time.time()
    for k in range(a.subsets):
        size = int(rng.integers(a.min_size, a.max_size + 1))
        idx = rng.choice(len(irs), size=min(size, len(irs)), replace=False)
        ms = step_ms([irs[i] for i in idx], data, a.steps)
        X.append(np.concatenate([feats[idx].sum(0), [1.0]]))
        y.append(ms / 1e3)
        print(f"subset {k}: {len(idx)} organisms  {ms:.3f} ms/step  ({time.time() - t0:.0f} s)", flush=True)
    X, y = np.array(X), np.array(y)
    from scipy.optimize import nnls
    # scale columns for conditioning
    sc = X.max(0)
    sc[sc == 0] = 1
    w, _ = nnls(X / sc, y)
    coef = w / sc
    pred = X @ coef
    rel = np.abs(pred - y) / y
    r2 = 1 - ((pred - y) ** 2).sum() / ((y - y.mean()) ** 2).sum()
    out = {"coef": {k: float(v) for k, v in zip(names, coef[:-1])}, "d_s": float(coef[-1]),
           "r2": float(r2), "mean_rel_err": float(rel.mean()), "max_rel_err": float(rel.max()),
           "subsets": int(len(y)), "source": "scripts/calibrate_cost.py on one MI355X (graph-replayed steps, B=750)"}
    print(json.dumps(out, indent=1), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    costs = np.array([CM.organism_time(ir, coef=out) for ir in irs])
    keys = [ir.arch_hash() for ir in irs]
    for R in (2, 4, 8):
        parts = lpt_partition(costs, R, keys)
        loads = np.array([costs[p].sum() + out["d_s"] for p in parts])
        print(f"LPT {R} ranks: predicted max/mean rank time {loads.max() / loads.mean():.4f} "
              f"(per-rank organisms {[len(p) for p in parts]})", flush=True)
    if a.measure_ranks > 1:
        R = a.measure_ranks
        parts = lpt_partition(costs, R, keys)
        meas = np.array([step_ms([irs[i] for i in p], data, a.steps) for p in parts])
        predicted = np.array([costs[p].sum() + out["d_s"] for p in parts]) * 1e3
        print(f"measured {R} shards: ms/step {np.round(meas, 3).tolist()} predicted {np.round(predicted, 3).tolist()} "
              f"measured max/mean {meas.max() / meas.mean():.4f}", flush=True)


if __name__ == "__main__":
    main()
