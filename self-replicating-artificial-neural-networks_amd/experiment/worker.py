"""Shard worker: the device work of one rank for one generation.

Reference: ``EvolutionaryExperimentWorker.run`` (evolutionary_experiment/logic/experiment_worker.py:
45-167).  For its shard of *trainable* organisms a rank builds one population engine, trains it
jointly (``fit``), evaluates on the test set and replicates each organism on its own rows.
Interpretation (validity / parameter count / overweight) is done by the replicated control plane
(:mod:`serann.experiment.population`), so the worker only sees trainable organisms.
"""
from __future__ import annotations

import hashlib
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from ..engine.base import TrainConfig, replication_image_rows
from ..genome.ir import OrganismIR


def replication_bits(outputs: np.ndarray) -> np.ndarray:
    """Sigmoid replication outputs -> offspring bits, ``round(clip(o, 0, 1))`` (experiment.py:206-209).

    A diverged organism (NaN / inf logits) has non-finite outputs.  The reference keeps NaN loci in the
    float genotype it stores (its DB reader parses 'nan'); offspring genotypes here travel bit-packed,
    so a non-finite locus is mapped explicitly: NaN -> 0, +inf -> 1, -inf -> 0 (docs/deviations.md)."""
    o = np.nan_to_num(np.asarray(outputs, np.float64), nan=0.0, posinf=1.0, neginf=0.0)
    return np.round(np.clip(o, 0, 1)).astype(np.uint8)


def organism_seed(random_seed: int, generation: int, organism_id: str) -> int:
    h = hashlib.blake2b(f"{random_seed}:{generation}:{organism_id}".encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & 0x7FFFFFFF


def make_engine(name: str, irs: Sequence[OrganismIR], seeds: Sequence[int], device, cfg: TrainConfig):
    if name == "torch":
        from ..engine.torch_engine import TorchPopulationEngine
        import torch
        dtype = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        return TorchPopulationEngine(irs, seeds, device=device, compute_dtype=dtype, cfg=cfg)
    if name == "hip":
        from ..engine.hip_engine import HipPopulationEngine
        return HipPopulationEngine(irs, seeds, device=device, cfg=cfg)
    raise ValueError(f"unknown engine {name!r}")


@dataclass
class ShardResult:
    indices: np.ndarray          # (n,) indices into the generation table
    metrics: np.ndarray          # (n, 4): val acc, train acc, test acc, replication mse
    offspring: np.ndarray        # (n, pool, L) uint8 {0,1} (rounded+clipped replication outputs)
    learning_time: float
    replication_time: float


class ShardWorker:
    def __init__(self, parameters: dict, data, engine: str = "torch", device="cpu",
                 train_cfg: Optional[TrainConfig] = None):
        self.params = parameters
        self.data = data
        self.engine_name = engine
        self.device = device
        self.cfg = train_cfg or TrainConfig(epochs=int(parameters["training_epochs"]),
                                            batch_size=int(parameters["training_batch_size"]))

    def run(self, indices: Sequence[int], ids: Sequence[str], genotypes: np.ndarray, irs: List[OrganismIR],
            num_replications: int, generation: int, random_seed: int,
            positions: Optional[Sequence[int]] = None, n_trainable: Optional[int] = None) -> ShardResult:
        """``positions``/``n_trainable``: the organisms' positions among *all* trainable organisms of
        the generation, which fixes their replication images independently of the partition (the
        reference's single-job layout, experiment_worker.py:140-160)."""
        n = len(indices)
        L = int(self.params["genotype_size"])
        if n == 0:
            return ShardResult(np.zeros(0, np.int32), np.zeros((0, 4)), np.zeros((0, num_replications, L), np.uint8),
                               0.0, 0.0)
        cfg = self.cfg
        cfg.seed = int(hashlib.blake2b(f"{random_seed}:{generation}:perm".encode(), digest_size=4).hexdigest(), 16)
        seeds = [organism_seed(random_seed, generation, i) for i in ids]
        engine = make_engine(self.engine_name, irs, seeds, self.device, cfg)
        try:
            fit = engine.fit(self.data, cfg)
            d = self.data
            test_acc = engine.evaluate(d.test_x, d.test_labels, d.test_g, cfg)
            learning_time = fit.learning_time

            offspring = np.zeros((n, num_replications, L), np.uint8)
            replication_time = 0.0
            if num_replications > 0:
                t0 = time.perf_counter()
                pos = list(range(n)) if positions is None else list(positions)
                total = (n if n_trainable is None else n_trainable) * num_replications
                images = [d.test_x[replication_image_rows(q, num_replications, total, len(d.test_x))]
                          for q in pos]
                outs = engine.replicate(np.asarray(genotypes, np.float32), images, cfg)
                for p, o in enumerate(outs):
                    offspring[p] = replication_bits(o)
                replication_time = time.perf_counter() - t0
        finally:
            engine.close()
        metrics = np.stack([fit.val_acc, fit.train_acc, test_acc, fit.val_mse], axis=1).astype(np.float64)
        return ShardResult(np.asarray(indices, np.int32), metrics, offspring, learning_time, replication_time)
