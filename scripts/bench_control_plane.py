#!/usr/bin/env python
"""Host cost of one generation outside the GPU work, at a given population size (default 1000, the
8-GPU bench): interpretation + partition, fertility / multinomial, statistics, SQLite writes,
selection + proofreading + decode.  The shard worker is replaced by an instant fake that returns
plausible metrics and offspring pools (parents' genotypes with ~1 % bit flips), so the numbers are
the serial work every rank (or rank 0) adds to a generation regardless of the GPU count.

    python scripts/bench_control_plane.py --pop 1000 --gens 4
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


class FakeWorker:
    def __init__(self, seed=0):
        self.rng = np.random.default_rng(seed)
        self.seconds = 0.0

    def run(self, indices, ids, genotypes, irs, num_replications, generation, random_seed, positions=None,
            n_trainable=None):
        from serann.experiment.worker import ShardResult
        t0 = time.perf_counter()
        n = len(indices)
        L = genotypes.shape[1] if n else 100
        metrics = np.stack([self.rng.uniform(0.5, 1.0, n), self.rng.uniform(0.5, 1.0, n),
                            self.rng.uniform(0.5, 1.0, n), self.rng.uniform(0.0, 0.2, n)], 1)
        off = np.repeat(np.asarray(genotypes, np.uint8)[:, None, :], num_replications, 1)
        flips = self.rng.random(off.shape) < 0.01
        off = np.where(flips, 1 - off, off).astype(np.uint8)
        self.seconds += time.perf_counter() - t0
        return ShardResult(np.asarray(indices, np.int32), metrics, off, 0.0, 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=1000)
    ap.add_argument("--gens", type=int, default=4)
    a = ap.parse_args()
    from serann.config import default_parameters
    from serann.experiment.experiment import Experiment
    from serann.experiment.runner import build_codec
    from serann.utils.db import ExperimentDB

    params = default_parameters("full_experiment")
    params["num_seranns"] = a.pop
    params["num_generations"] = a.gens
    codec = build_codec(params, "table", seed=0)
    enc = np.random.default_rng(0).integers(0, 2, (70000, int(params["genotype_size"]))).astype(np.uint8)
    tmp = tempfile.mkdtemp(prefix="serann_cp_")
    db = ExperimentDB(os.path.join(tmp, f"{uuid.uuid4()}.sqlite"))
    worker = FakeWorker()
    exp = Experiment("cp", enc, worker, db, params, codec, random_seed=79375, verbose=False)
    t0 = time.perf_counter()
    hist = exp.execute()
    total = time.perf_counter() - t0
    for h in hist:
        print(json.dumps({"generation": h["generation"], "seconds": round(h["seconds"], 4),
                          "phases": {k: round(v, 4) for k, v in h["phases"].items()}}))
    print(json.dumps({"pop": a.pop, "gens": len(hist), "seconds_per_generation": total / max(1, len(hist)),
                      "fake_worker_seconds": worker.seconds}))


if __name__ == "__main__":
    main()
