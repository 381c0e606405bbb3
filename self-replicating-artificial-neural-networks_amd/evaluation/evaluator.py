"""Retrospective fertility / mutation-rate evaluation (reference: serann_evaluation/logic.py:17-272).

``SerannEvaluator.evaluate`` for one genotype:
 1. decode to source; ``loss_balance`` parsed with the reference regex (logic.py:165);
 2. train E = ``num_evaluations`` identical replicas jointly (5 epochs, batch 750, validation 5 %)
    -> E validation accuracies;
 3. replicate R = ``replications_per_evaluation`` offspring per replica on the first R test images;
 4. round / clip, probabilistic proofreading, decode;
 5. per replica: offspring-survival histogram {valid: count} (validity = builds, cached by source)
    and mutation-rate histogram {rate: count}.

The E replicas are one *homogeneous* population engine (every grouped launch then holds E copies of
the same problem).  ``evaluate_many`` batches several genotypes into one engine to fill the GPU.

Reference quirks: the mutation-rate window ``fixed[i:i+R]`` (item 1) is reproduced only
with ``strict_reference=True`` -- by default replica i uses its own rows ``[i*R, (i+1)*R)``; cached
invalid sources are not re-built (item 2).
"""
from __future__ import annotations

import re
import time
from collections import Counter
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..engine.base import TrainConfig
from ..experiment.population import InterpretCache
from ..experiment.worker import make_engine, organism_seed

LB_REGEX = re.compile(r"loss_balance *= *([0-9]+\.[0-9]+?)(\s|$)")

EMPTY = {"classification_accuracy": np.nan, "offspring_survival": {}, "mutation_rate": {}}


def genotype_key(genotype) -> str:
    """Stable identity of a genotype: its bits as a hex string (NaN / non-binary loci kept distinct)."""
    g = np.asarray(genotype, np.float64)
    if np.all((g == 0) | (g == 1)):
        return np.packbits(g.astype(np.uint8)).tobytes().hex()
    return g.tobytes().hex()


def probabilistic_proofreading(parent, offspring, ec_factor: float, rng: np.random.RandomState):
    """Revert a random fraction ``ec_factor`` of the loci that differ from the parent (common/logic.py:6-14)."""
    offspring = np.array(offspring, copy=True)
    rows, cols = np.where(offspring != parent)
    fixed = rng.permutation(len(rows))[:int(ec_factor * len(rows))]
    rows, cols = rows[fixed], cols[fixed]
    offspring[rows, cols] = np.asarray(parent)[cols]
    return offspring


class SerannEvaluator:
    def __init__(self, experiment_params: dict, data, codec, num_evaluations: int = 50,
                 replications_per_evaluation: int = 100, engine: str = "torch", device="cpu",
                 train_cfg: Optional[TrainConfig] = None, seed: int = 0, strict_reference: bool = False,
                 max_parameters: float = float("inf")):
        self.params = experiment_params
        self.data = data
        self.codec = codec
        self.E = int(num_evaluations)
        self.R = int(replications_per_evaluation)
        self.engine = engine
        self.device = device
        self.cfg = train_cfg or TrainConfig(epochs=int(experiment_params["training_epochs"]),
                                            batch_size=int(experiment_params["training_batch_size"]))
        self.rng = np.random.RandomState(seed)
        self.seed = seed
        self.strict = strict_reference
        self.max_parameters = max_parameters
        self.cache = InterpretCache(experiment_params.get("classification_image_dimensions", (28, 28)),
                                    int(experiment_params["genotype_size"]),
                                    int(experiment_params["num_classification_classes"]))
        self._validity: Dict[str, int] = {}
        # wall seconds per phase, accumulated over evaluate_many calls (scripts/bench_evaluation.py)
        self.timings: Dict[str, float] = {"engine_init": 0.0, "fit": 0.0, "replicate": 0.0, "host_post": 0.0}

    def is_valid_serann(self, source_code: str) -> int:
        v = self._validity.get(source_code)
        if v is None:
            v = int(self.cache(source_code).ok)
            self._validity[source_code] = v
        return v

    def evaluate(self, genotype, source_code: Optional[str] = None, loss_balance: Optional[float] = None) -> dict:
        return self.evaluate_many([genotype], [source_code], [loss_balance])[0]

    def evaluate_many(self, genotypes: Sequence, source_codes: Optional[Sequence] = None,
                      loss_balances: Optional[Sequence] = None) -> List[dict]:
        n = len(genotypes)
        genotypes = [np.asarray(g).astype(int) for g in genotypes]
        source_codes = list(source_codes) if source_codes is not None else [None] * n
        loss_balances = list(loss_balances) if loss_balances is not None else [None] * n
        need = [i for i in range(n) if source_codes[i] is None]
        if need:
            dec = self.codec.decode_to_string(np.stack([genotypes[i] for i in need]))
            for i, s in zip(need, dec):
                source_codes[i] = s
        results: List[Optional[dict]] = [None] * n
        irs, owners = [], []
        for i in range(n):
            if loss_balances[i] is None:
                m = LB_REGEX.search(source_codes[i])
                if m is None:
                    results[i] = dict(EMPTY)
                    continue
            r = self.cache(source_codes[i])
            if not r.ok or r.parameters_count > self.max_parameters:
                results[i] = dict(EMPTY)
                continue
            for e in range(self.E):
                irs.append(r.ir)
                owners.append((i, e))
        if irs:
            # keyed on the genotype itself (not its position in this batch), so a genotype gets the same
            # replica initialisations however run_many batches / de-duplicates / shards the sample
            keys = {i: genotype_key(genotypes[i]) for i, _ in owners}
            seeds = [organism_seed(self.seed, keys[i], f"eval{e}") for i, e in owners]
            t0 = time.perf_counter()
            eng = make_engine(self.engine, irs, seeds, self.device, self.cfg)
            t1 = time.perf_counter()
            try:
                fit = eng.fit(self.data, self.cfg)
                t2 = time.perf_counter()
                imgs = [self.data.test_x[:self.R]] * len(irs)
                gens = np.stack([genotypes[i] for i, _ in owners]).astype(np.float32)
                outs = eng.replicate(gens, imgs, self.cfg)
                t3 = time.perf_counter()
            finally:
                eng.close()
            self.timings["engine_init"] += t1 - t0
            self.timings["fit"] += t2 - t1
            self.timings["replicate"] += t3 - t2
            t4 = time.perf_counter()
            by_sample: Dict[int, list] = {}
            for k, (i, e) in enumerate(owners):
                by_sample.setdefault(i, []).append((fit.val_acc[k], outs[k]))
            ec = float(self.params.get("error_correction_probability", 0))
            for i, items in by_sample.items():
                g = genotypes[i]
                acc = [float(a) for a, _ in items]
                reps = np.concatenate([o for _, o in items], 0)                  # (E*R, L)
                offspring = np.round(np.clip(reps, 0, 1))
                fixed = probabilistic_proofreading(g, offspring, ec, self.rng)
                srcs = self.codec.decode_to_string(fixed)
                survival, mutation = [], []
                for e in range(self.E):
                    hist: Dict[int, int] = {}
                    for j in range(self.R):
                        v = self.is_valid_serann(srcs[e * self.R + j])
                        hist[v] = hist.get(v, 0) + 1
                    survival.append(hist)
                    rows = fixed[e:e + self.R] if self.strict else fixed[e * self.R:(e + 1) * self.R]
                    rates = np.sum(rows != g, axis=1) / len(g)
                    mutation.append(dict(Counter(rates.tolist())))
                results[i] = {"classification_accuracy": acc, "mutation_rate": mutation,
                              "offspring_survival": survival}
            self.timings["host_post"] += time.perf_counter() - t4
        return results


class SerannEvaluationWorker(SerannEvaluator):
    """Evaluator + genotype-hex keyed result cache (serann_evaluation/logic.py:234-272)."""

    def __init__(self, *args, evaluation_cache: bool = True, **kwargs):
        super().__init__(*args, **kwargs)
        self._evaluations_cache: Optional[dict] = {} if evaluation_cache else None

    def run_many(self, rows) -> List[tuple]:
        """rows: list of (serann_id, row dict with genotype, genotype_hex, is_valid, is_overweight)."""
        out: Dict[str, dict] = {}
        todo = []
        for sid, row in rows:
            key = row["genotype_hex"]
            if self._evaluations_cache is not None and key in self._evaluations_cache:
                out[sid] = self._evaluations_cache[key]
            elif not bool(row["is_valid"]) or bool(row["is_overweight"]):
                out[sid] = dict(EMPTY)
            else:
                todo.append((sid, row))
        # de-duplicate genotypes inside the batch
        uniq = {}
        for sid, row in todo:
            uniq.setdefault(row["genotype_hex"], (sid, row))
        if uniq:
            keys = list(uniq)
            res = self.evaluate_many([np.asarray(uniq[k][1]["genotype"]) for k in keys])
            for k, r in zip(keys, res):
                if self._evaluations_cache is not None:
                    self._evaluations_cache[k] = r
            for sid, row in todo:
                out[sid] = self._evaluations_cache[row["genotype_hex"]] if self._evaluations_cache is not None \
                    else res[keys.index(row["genotype_hex"])]
        if self._evaluations_cache is not None:
            for sid, row in rows:
                self._evaluations_cache.setdefault(row["genotype_hex"], out[sid])
        return [(sid, out[sid]) for sid, _ in rows]

    def run(self, serann_id, serann_info) -> tuple:
        return self.run_many([(serann_id, serann_info)])[0]

    def handle_update(self, update_data: dict):
        if self._evaluations_cache is not None:
            self._evaluations_cache.update(update_data)
