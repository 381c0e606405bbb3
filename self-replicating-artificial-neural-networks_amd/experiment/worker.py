"""Shard worker: the device work of one rank for one generation.

Reference: ``EvolutionaryExperimentWorker.run`` (evolutionary_experiment/logic/experiment_worker.py:
45-167).  For its shard of *trainable* organisms a rank builds one population engine, trains it
jointly (``fit``), evaluates on the test set and replicates each organism on its own rows.
Interpretation (validity / parameter count / overweight) is done by the replicated control plane
(:mod:`serann.experiment.population`), so the worker only sees trainable organisms.  Shards larger
than the device budget train in waves with an out-of-memory fallback (:mod:`serann.experiment.capacity`,
replacing the reference's 112-organism jobs and half-batch retry, experiment_worker.py:121-126).
"""
from __future__ import annotations

import dataclasses
import hashlib
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np

from ..engine.base import TrainConfig, replication_image_rows
from ..genome.ir import OrganismIR
from . import capacity


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
    packed: object               # (n, pool, ceil(L / 8)) uint8 offspring bits (numpy.packbits order):
                                 # a device tensor straight from the HIP replication epilogue, or numpy
    learning_time: float
    replication_time: float
    L: int = 0

    @property
    def offspring(self) -> np.ndarray:
        """(n, pool, L) uint8 {0,1} (rounded + clipped replication outputs), unpacked on the host."""
        p = self.packed
        if not isinstance(p, np.ndarray):
            p = p.detach().cpu().numpy()
        return np.unpackbits(np.asarray(p, np.uint8), axis=-1)[..., :self.L]


class ShardWorker:
    def __init__(self, parameters: dict, data, engine: str = "torch", device="cpu",
                 train_cfg: Optional[TrainConfig] = None, max_per_wave: Optional[int] = None,
                 log: Optional[Callable[[str], None]] = None):
        self.params = parameters
        self.data = data
        self.engine_name = engine
        self.device = device
        self.cfg = train_cfg or TrainConfig(epochs=int(parameters["training_epochs"]),
                                            batch_size=int(parameters["training_batch_size"]))
        self.max_per_wave = max_per_wave
        self.log = log or (lambda m: print(m, flush=True))
        self.last_waves: List[List[int]] = []        # (introspection: tests, perf log)

    def steps_per_generation(self) -> int:
        """Training steps of one generation (epochs x steps per epoch of the training split): the factor between
        the cost model's seconds per step and a shard's learning seconds."""
        n = int(getattr(self.data, "n_train", 0) or 0)
        if n <= 0:
            return 0
        return int(self.cfg.epochs) * int(self.cfg.steps_per_epoch(self.cfg.split(n)))

    def run(self, indices: Sequence[int], ids: Sequence[str], genotypes: np.ndarray, irs: List[OrganismIR],
            num_replications: int, generation: int, random_seed: int,
            positions: Optional[Sequence[int]] = None, n_trainable: Optional[int] = None) -> ShardResult:
        """``positions``/``n_trainable``: the organisms' positions among *all* trainable organisms of
        the generation, which fixes their replication images independently of the partition (the
        reference's single-job layout, experiment_worker.py:140-160).

        The shard is trained in one engine when it fits the rank's device budget, else in waves
        (:mod:`serann.experiment.capacity`); an out-of-memory error splits a wave and retries."""
        n = len(indices)
        L = int(self.params["genotype_size"])
        nbytes = (L + 7) // 8
        if n == 0:
            return ShardResult(np.zeros(0, np.int32), np.zeros((0, 4)), np.zeros((0, num_replications, nbytes), np.uint8),
                               0.0, 0.0, L)
        cfg = self.cfg
        cfg.seed = int(hashlib.blake2b(f"{random_seed}:{generation}:perm".encode(), digest_size=4).hexdigest(), 16)
        seeds = [organism_seed(random_seed, generation, i) for i in ids]
        d = self.data
        pos = list(range(n)) if positions is None else list(positions)
        total = (n if n_trainable is None else n_trainable) * num_replications
        genotypes = np.asarray(genotypes, np.float32)

        budget = capacity.device_budget(self.device)
        sizes = [capacity.organism_device_bytes(ir, cfg.batch_size, min(num_replications, cfg.batch_size))
                 for ir in irs]
        waves = capacity.plan_waves(sizes, budget, self.max_per_wave)
        self.last_waves = []
        if len(waves) > 1:
            self.log(f"shard of {n} organisms (~{sum(sizes) / 1e9:.1f} GB) trained in {len(waves)} waves "
                     f"(budget {budget / 1e9:.1f} GB)" if budget else f"shard of {n} organisms in {len(waves)} waves")

        metrics = np.full((n, 4), np.nan)
        packed = None            # device tensor (HIP epilogue) or numpy, [n][pool][nbytes]
        times = [0.0, 0.0]

        # host-side phases of the shard (seconds, summed over waves): where a generation's time goes
        # besides the training loop itself (``learning_time``)
        ph = self.last_phases = dict.fromkeys(("construct", "alloc", "plan", "fit", "test_eval", "replicate", "close"),
                                              0.0)

        def run_wave(members: List[int], batch: Optional[int]):
            wcfg = cfg if batch is None else dataclasses.replace(cfg, batch_size=int(batch))
            tc = time.perf_counter()
            engine = make_engine(self.engine_name, [irs[i] for i in members], [seeds[i] for i in members],
                                 self.device, wcfg)
            ph["construct"] += time.perf_counter() - tc
            try:
                tc = time.perf_counter()
                fit = engine.fit(d, wcfg)
                ph["fit"] += time.perf_counter() - tc
                ex = getattr(fit, "extra", None) or {}
                ph["plan"] += float(ex.get("plan_s", 0.0))          # includes the buffer allocation
                ph["alloc"] += float(ex.get("alloc_s", 0.0))
                tc = time.perf_counter()
                test_acc = engine.evaluate(d.test_x, d.test_labels, d.test_g, wcfg)
                ph["test_eval"] += time.perf_counter() - tc
                outs, rt = None, 0.0
                if num_replications > 0:
                    t0 = time.perf_counter()
                    images = [d.test_x[replication_image_rows(pos[i], num_replications, total, len(d.test_x))]
                              for i in members]
                    if hasattr(engine, "replicate_packed"):
                        outs = engine.replicate_packed(genotypes[members], images, wcfg)   # device, packed
                    else:
                        outs = np.packbits(np.stack([replication_bits(o) for o in
                                                     engine.replicate(genotypes[members], images, wcfg)]), axis=-1)
                    rt = time.perf_counter() - t0
                    ph["replicate"] += rt
            finally:
                tc = time.perf_counter()
                engine.close()
                ph["close"] += time.perf_counter() - tc
            return members, fit, test_acc, outs, fit.learning_time, rt

        def on_fail(members: List[int]):
            return members, None, None, None, 0.0, 0.0

        for w in waves:
            for members, fit, test_acc, outs, lt, rt in capacity.run_with_fallback(
                    w, run_wave, cfg.batch_size, self.device, self.log, on_fail):
                self.last_waves.append(list(members))
                times[0] += lt
                times[1] += rt
                if fit is None:
                    continue                               # did not fit even at half batch: NaN metrics
                metrics[members] = np.stack([fit.val_acc, fit.train_acc, test_acc, fit.val_mse], axis=1)
                if outs is not None and len(members):
                    if packed is None:
                        packed = (outs.new_zeros((n, num_replications, nbytes)) if not isinstance(outs, np.ndarray)
                                  else np.zeros((n, num_replications, nbytes), np.uint8))
                    packed[members] = outs
        if packed is None:
            packed = np.zeros((n, num_replications, nbytes), np.uint8)
        return ShardResult(np.asarray(indices, np.int32), metrics.astype(np.float64), packed, times[0], times[1], L)
