"""Evaluation driver: samplers + ``SampleDeepEvaluator`` (reference: serann_evaluation/run_evaluation.py:22-197,
serann_evaluation/logic.py:17-87).

Samplers (registered by name through a metaclass, as in the reference):
``mutants`` (mutants interleaved with their parents), ``unique_genotypes``, ``unique_source_codes``,
``general`` (every ``generation_step``-th generation plus generation 1).

SPMD instead of a job pool: the remaining sample ids are split round-robin over the ranks; ranks work
in rounds of ``batch`` samples (one multi-genotype engine per round) and after every round all ranks
all-gather their results -- rank 0 records them and pickles every 100 results, every rank merges them
into its genotype cache (the reference's shared-cache broadcast, M4).
"""
from __future__ import annotations

import os
import pickle
import shutil
import time
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import pandas as pd

from ..parallel.comm import Comm, LocalComm
from ..utils.faults import maybe_inject_evaluation

SAMPLERS: Dict[str, type] = {}


class MetaSampler(type):
    def __new__(mcs, name, bases, attrs):
        cls = super().__new__(mcs, name, bases, attrs)
        if name != "SamplerInterface":
            SAMPLERS[attrs["name"]] = cls
        return cls


class SamplerInterface(metaclass=MetaSampler):
    def __init__(self, seed: Optional[int] = None):
        self.rng = np.random.RandomState(seed)

    def sample(self, df: pd.DataFrame, parameters: dict) -> pd.Index:
        raise NotImplementedError


class MutantsSampler(SamplerInterface):
    name = "mutants"

    def sample(self, df, parameters):
        mask = df["parent_id"].notna() & df["parent_id"].isin(df.index) & \
            df["genotype_hex"].ne(df["parent_genotype_hex"])
        pool = df[mask]
        n = min(int(parameters["total_samples"]), len(pool)) if parameters["total_samples"] > -1 else len(pool)
        sample = pool.sample(n, random_state=self.rng)
        sample = sample.sample(frac=1, random_state=self.rng).assign(temp_index=np.arange(len(sample)))
        parents = df.loc[sample["parent_id"]].assign(temp_index=np.arange(len(sample)))
        return pd.concat([sample, parents]).sort_values("temp_index", kind="stable").index


class UniqueGenotypesSampler(SamplerInterface):
    name = "unique_genotypes"

    def sample(self, df, parameters):
        u = df.sample(frac=1, random_state=self.rng).drop_duplicates(subset=["genotype_hex"])
        return u.iloc[:parameters["total_samples"]].index if parameters["total_samples"] > -1 else u.index


class UniqueSourceCodesSampler(SamplerInterface):
    name = "unique_source_codes"

    def sample(self, df, parameters):
        u = df.sample(frac=1, random_state=self.rng).drop_duplicates(subset=["source_code"])
        return u.iloc[:parameters["total_samples"]].index if parameters["total_samples"] > -1 else u.index


class GeneralSampler(SamplerInterface):
    name = "general"

    def sample(self, df, parameters):
        step = int(parameters["generation_step"])
        mask = ((df["generation"] % step == 0) & (df["generation"] != 0)) | (df["generation"] == 1)
        sub = df[mask]
        k = int(parameters["samples_per_generation"])
        if k > 0:
            parts = [g.sample(min(k, len(g)), random_state=self.rng) for _, g in sub.groupby("generation")]
            sample = pd.concat(parts) if parts else sub.iloc[:0]
        else:
            n = min(int(parameters["total_samples"]), len(sub))
            sample = sub.sample(n, random_state=self.rng)
        return sample.sample(frac=1, random_state=self.rng).index


class SampleDeepEvaluator:
    def __init__(self, experiment_df: pd.DataFrame, output_path: str, sample_ids, worker, comm: Optional[Comm] = None,
                 shared_cache: bool = True, batch: int = 4, log=print, save_every: int = 100):
        self.comm = comm or LocalComm()
        self._exp_df = experiment_df
        self._output_path = str(output_path)
        self._shared = shared_cache
        self.worker = worker
        self.batch = max(1, int(batch))
        self.save_every = max(1, int(save_every))       # results between pickles (reference: 100)
        self.log = log if self.comm.is_root else (lambda *a, **k: None)
        sample_ids = list(pd.Index(sample_ids).drop_duplicates())
        if Path(self._output_path).is_file():
            self.log("Resuming existing SeRANNs sample evaluation")
            with open(self._output_path, "rb") as f:          # written by this class (our own file)
                sample = pickle.load(f)
            self._use_existing_sample(sample)
        else:
            self.log("Sampling SeRANNs for evaluation")
            self._sample_metadata = self._exp_df.loc[sample_ids]
            self._results = {i: {} for i in sample_ids}

    def _use_existing_sample(self, sample: dict):
        cache = {}
        for sid, v in sample.items():
            if len(v) > 0 and sid in self._exp_df.index:
                cache[self._exp_df.at[sid, "genotype_hex"]] = v
        self.worker.handle_update(cache)
        self._results = sample
        self._sample_metadata = self._exp_df.loc[[s for s in sample if s in self._exp_df.index]]
        if self.comm.is_root:
            path = Path(self._output_path)
            shutil.copy(path, path.with_name(path.stem + "_backup.pkl"))

    @property
    def results(self):
        return self._results

    def run(self):
        comm = self.comm
        remaining = [i for i, r in self._results.items() if len(r) == 0]
        mine = remaining[comm.rank::comm.world_size]
        rounds = -(-max(len(remaining[r::comm.world_size]) for r in range(comm.world_size)) // self.batch) \
            if remaining else 0
        done = 0
        durations = []
        t_run = time.perf_counter()
        for k in range(rounds):
            t0 = time.perf_counter()
            chunk = mine[k * self.batch:(k + 1) * self.batch]
            rows = []
            for sid in chunk:
                r = self._sample_metadata.loc[sid]
                rows.append((sid, {"genotype": r["genotype"], "genotype_hex": r["genotype_hex"],
                                   "is_valid": r["is_valid"], "is_overweight": r["is_overweight"]}))
            out = self.worker.run_many(rows) if rows else []
            gathered = comm.allgather_object(out)
            for part in gathered:
                for sid, res in part:
                    if self._shared:
                        self.worker.handle_update({self._exp_df.at[sid, "genotype_hex"]: res})
                    self._results[sid] = {"classification_accuracy": res["classification_accuracy"],
                                          "mutation_rate": res["mutation_rate"],
                                          "offspring_survival": res["offspring_survival"]}
                    done += 1
            durations.append((time.perf_counter() - t0) / max(1, sum(len(p) for p in gathered)))
            avg = float(np.mean(durations[-200:]))
            self.log(f"{done}/{len(remaining)} jobs done. Average evaluation time: {int(avg) // 60:02d}:"
                     f"{int(avg) % 60:02d}. ({avg:.3f} s per genotype, {time.perf_counter() - t_run:.1f} s elapsed)")
            se = self.save_every
            if comm.is_root and (done // se != (done - sum(len(p) for p in gathered)) // se or k == rounds - 1):
                self.log("Saving to disk.")
                self.save()
                maybe_inject_evaluation(sum(1 for r in self._results.values() if len(r)), comm.rank)
        if comm.is_root and rounds == 0:
            self.save()
        return self._results

    def save(self):
        Path(self._output_path).parent.mkdir(parents=True, exist_ok=True)
        tmp = self._output_path + ".tmp"
        with open(tmp, "wb") as f:
            pickle.dump(self._results, f)
        os.replace(tmp, self._output_path)
