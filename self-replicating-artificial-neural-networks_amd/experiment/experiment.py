"""The evolutionary generation loop (reference: evolutionary_experiment/logic/experiment.py:23-329).

SPMD structure: every rank runs this loop with the same seeded RNG over the same generation table
(replicated control plane); only the training of organisms is sharded (LPT partition), and one
packed all-gather per generation brings metrics and bit-packed offspring pools to every rank.
Rank 0 alone writes the SQLite DB and prints.

Per generation (experiment.py:51-101):
 1. interpret sources -> validity, parameter count, overweight flag;
 2. learn + replicate (sharded);
 3. fertility = val_acc ** selection_pressure, relative fertility normalised (NaN -> 0);
 4. offspring counts ~ Multinomial(num_seranns, relative fertility);
 5. layer counts, generation statistics, DB rows;
 6. stop if no valid SeRANN remains;
 7. offspring selection (random | best) + probabilistic proofreading, decode, distances;
 8. pool size = max(num_offspring) * offspring_pool_size_factor.

Fixes relative to the reference (documented in docs/deviations.md): ids come from the seeded RNG
(reproducible), row order is the deterministic table order (not job-completion order), the
replication step is O(P * pool), a parent with more offspring than its pool samples the excess with
replacement (the reference crashes), and resume is exact via ``resume_state``.
"""
from __future__ import annotations

import json
import time
import uuid
from datetime import datetime
from typing import Callable, Dict, List, Optional

import numpy as np
import pandas as pd

from ..genome.interpreter import layer_counts
from ..parallel.comm import Comm, LocalComm, pack_header, unpack_header, unpack_results
from ..parallel.partition import RankSpeedModel, lpt_partition
from ..utils.faults import GenerationWatchdog, job_scale, maybe_inject
from ..utils.levenshtein import levenshtein_batch
from ..utils.stats import fertility, genotype_stats, source_code_stats
from ..utils.trace import PhaseTimer, phase
from .population import InterpretCache, plan_generation
from .worker import ShardWorker

MODEL_INFO_COLUMNS = ["parameters_count", "loss_balance", "is_valid", "is_overweight",
                      "classification_validation_accuracy", "classification_training_accuracy",
                      "classification_test_accuracy", "replication_mse"]


def hamming(a, b):
    return np.not_equal(a, b).sum(axis=-1) / np.shape(a)[-1]


class Experiment:
    def __init__(self, experiment_id: str, serann_dataset: np.ndarray, worker: ShardWorker, experiment_db,
                 parameters: dict, codec, comm: Optional[Comm] = None, start_generation: int = 0,
                 random_seed: int = 0, strict_reference: bool = False, verbose: bool = True,
                 perf_log: Optional[str] = None, job_timeout: Optional[float] = None):
        self._id = experiment_id
        self._serann_dataset = serann_dataset
        self._worker = worker
        self._db = experiment_db
        self._parameters = parameters
        self._codec = codec
        self._comm = comm or LocalComm()
        self._start_generation = start_generation
        self._random_seed = int(random_seed)
        self._rng = np.random.RandomState(self._random_seed)
        self._strict = strict_reference
        self._verbose = verbose and self._comm.is_root
        self._perf_log = perf_log
        self._cache = InterpretCache(parameters.get("classification_image_dimensions", (28, 28)),
                                     int(parameters["genotype_size"]),
                                     int(parameters["num_classification_classes"]))
        self.history: List[dict] = []
        # per-rank speed factors learned from measured shard times (replicated: every rank updates the same)
        self._speeds = RankSpeedModel(self._comm.world_size)
        if job_timeout is None:
            # the reference pool's per-job timeout (config.py:7), armed by default only where a stall is
            # plausible and recoverable: the GPU engine, or a run under the supervising launcher.  A slow
            # but healthy CPU run is never killed by it.
            from ..cli.launch import CHILD_ENV
            from ..config import experiment_config
            import os
            gpu = str(getattr(worker, "engine_name", "")) == "hip"
            job_timeout = float(experiment_config["worker_pool_job_timeout"]) if (gpu or os.environ.get(CHILD_ENV)) \
                else 0.0
        # per-generation watchdog, scaled to the rank's shard once the partition is known
        self._watchdog = GenerationWatchdog(job_timeout, self._comm.rank)
        if self._comm.is_root and self._db is not None:
            self._db.save_execution_info(datetime.now(), self._parameters)

    # ------------------------------------------------------------------------------------------
    def log(self, *a):
        if self._verbose:
            print(*a, flush=True)

    def _new_ids(self, n: int) -> List[str]:
        # one draw of 16 n bytes: RandomState.bytes draws whole 32-bit words, so this is the same byte
        # stream (and RNG state afterwards) as n draws of 16 bytes
        raw = self._rng.bytes(16 * n) if n > 0 else b""
        return [str(uuid.UUID(bytes=raw[16 * k:16 * k + 16], version=4)) for k in range(n)]

    def execute(self, max_generations: Optional[int] = None,
                on_generation: Optional[Callable[[int, dict], None]] = None):
        p = self._parameters
        self.log(f"Experiment {self._id} has started")
        self.log(f"Using {self._comm.world_size} GPU workers")
        current, offspring_pool_size = self._get_first_generation()
        self.log("Initial offspring pool size:", offspring_pool_size)
        end = int(p["num_generations"])
        if max_generations is not None:
            end = min(end, self._start_generation + max_generations)
        for generation_number in range(self._start_generation, end):
            generation_start_time = datetime.now()
            t0 = time.perf_counter()
            self.log(f"### Generation {generation_number} execution has started ###")
            timer = PhaseTimer()
            current["experiment_id"] = self._id
            current["generation"] = generation_number
            current["num_offspring"] = 0

            self.log("Starting training and replication")
            self._watchdog.arm(f"generation {generation_number}")
            try:
                maybe_inject(generation_number, self._comm.rank)      # SERANN_FAULT_INJECT (recovery tests)
                with phase("learn_and_replicate", timer):
                    models_info, offspring_by_id, times = self._learn_and_replicate(current, offspring_pool_size,
                                                                                   generation_number)
            finally:
                self._watchdog.disarm()
            current = current.join(models_info)

            self.log("Calculating fecundity scores")
            absolute, relative = fertility(current["classification_validation_accuracy"].to_numpy(),
                                           p["selection_pressure"])
            current["absolute_fertility"], current["relative_fertility"] = absolute, relative

            self.log("Sampling offspring counts")
            if current["is_valid"].sum() > 0 and relative.sum() > 0:
                current["num_offspring"] = self._rng.multinomial(int(p["num_seranns"]), relative)

            valid_serann = current[current["is_valid"] & ~current["is_overweight"].astype(bool)]
            self.log("Extracting source codes statistics")
            stats = pd.DataFrame([layer_counts(s) for s in valid_serann["source_code"]], index=valid_serann.index,
                                 columns=["classification_layers", "replication_layers", "merged_layers"])
            current = current.join(stats, how="left")

            t_stats = time.perf_counter()
            with phase("statistics", timer):
                generation_info = self._generation_statistics(current, generation_number, times,
                                                              generation_start_time)
            if self._comm.is_root and self._db is not None:
                with phase("db_write", timer):
                    self.log("Saving generation information to the experiment DB")
                    self._db.save_generation_info(generation_info)
                    self.log("Saving SeRANN records to the experiment DB")
                    self._db.save_seranns_info(current)
            t_db = time.perf_counter()

            record = dict(generation=generation_number, seconds=None, learning_time=float(np.mean(times["learning_times"] or [0])),
                          replication_time=float(np.mean(times["replication_times"] or [0])),
                          valid=int(len(valid_serann)), population=int(len(current)),
                          train_tflop=times["train_flops"] / 1e12,
                          mean_val_acc=float(np.nanmean(current["classification_validation_accuracy"]))
                          if len(valid_serann) else float("nan"),
                          stats_db_seconds=t_db - t_stats)
            wp = getattr(self._worker, "last_phases", None)
            if wp:
                record["shard_phases"] = {k: round(v, 4) for k, v in wp.items()}      # this rank's shard
            record["ranks"] = times.get("ranks", [])
            record["allgather_s"] = round(float(times.get("allgather_s", 0.0)), 5)
            record["allgather_bytes"] = int(times.get("allgather_bytes", 0))
            # max / mean learning seconds over the ranks that trained anything (1.0 at world size 1)
            ms = [v for v in times["rank_measured_s"] if v > 0]
            record["rank_imbalance"] = max(ms) / (sum(ms) / len(ms)) if ms else float("nan")
            record["rank_factors"] = times["rank_factors"]

            if len(valid_serann) == 0:
                self.log("No valid SeRANNs left! stopping...")
                record["seconds"] = time.perf_counter() - t0
                self._finish_record(record, on_generation)
                break

            self.log("Applying offspring selection")
            with phase("selection", timer):
                next_generation = self._select_offspring(current, offspring_by_id)
            self.log(f"Generation {generation_number} execution is done")
            offspring_pool_size = int(current["num_offspring"].max() * p["offspring_pool_size_factor"])
            self.log("Offspring pool size was updated to:", offspring_pool_size)
            if self._comm.is_root and self._db is not None:
                self._db.save_resume_state(generation_number, {
                    "next_generation": next_generation, "pool_size": offspring_pool_size,
                    "rng": self._rng.get_state(), "random_seed": self._random_seed})
            current = next_generation
            record["seconds"] = time.perf_counter() - t0
            record["phases"] = timer.reset()
            lr = record["phases"].get("learn_and_replicate")
            if lr:
                record["achieved_tflops"] = record["train_tflop"] / lr      # model FLOPs / learn+replicate time
            self._print_generation_time(record["seconds"])
            self._finish_record(record, on_generation)
        return self.history

    def _finish_record(self, record, on_generation):
        self.history.append(record)
        if self._perf_log and self._comm.is_root:
            with open(self._perf_log, "a") as f:
                f.write(json.dumps(record) + "\n")
        if on_generation is not None:
            on_generation(record["generation"], record)

    def _print_generation_time(self, seconds: float):
        s = int(seconds)
        self.log(f"\033[1mGeneration execution time: {s // 3600:02d}:{(s // 60) % 60:02d}:{s % 60:02d} "
                 f"({seconds:.2f} s)\033[0m")

    # ------------------------------------------------------------------------------------------
    def _get_first_generation(self):
        p = self._parameters
        if self._start_generation > 0:
            return self._load_last_generation_from_db()
        ancestor = p.get("ancestor_genotype")
        n = int(p["num_seranns"])
        if ancestor is None:
            sample = self._rng.randint(0, len(self._serann_dataset), n)
            genotypes = [np.asarray(self._serann_dataset[s]) for s in sample]
        else:
            genotypes = [np.asarray(ancestor) for _ in range(n)]
        ids = self._new_ids(n)
        current = pd.DataFrame({"genotype": genotypes}, index=pd.Index(ids, name="id"))
        current["source_code"] = self._codec.decode_to_string(np.stack(genotypes))
        current["parent_id"] = None
        current["genotype_euclidean_distance_from_parent"] = np.nan
        current["genotype_hamming_distance_from_parent"] = np.nan
        current["source_code_levenshtein_distance_from_parent"] = np.nan
        return current, int(p["initial_offspring_pool_size"])

    def _load_last_generation_from_db(self):
        """Exact resume from ``resume_state`` when present; otherwise the reference behaviour:
        retrain + re-replicate the last stored generation (experiment.py:119-135)."""
        last = self._start_generation - 1
        state = None
        if self._comm.is_root and self._db is not None:
            state = self._db.get_resume_state(last)
        state = self._comm.broadcast_object(state)
        if state is not None:
            self._rng.set_state(state["rng"])
            self.log("Resuming from the stored resume state")
            return state["next_generation"], int(state["pool_size"])
        last_generation = self._comm.broadcast_object(
            self._db.get_serann_by_generation(last) if self._comm.is_root else None)
        valid_mask = (last_generation["is_valid"] == True) & (last_generation["is_overweight"] == False)  # noqa
        valid = last_generation[valid_mask]
        if len(valid) == 0 or valid["num_offspring"].sum() == 0:
            raise RuntimeError("No valid SeRANNs left in the last generation!")
        self.log("Retraining and replicating the last generation")
        pool_size = int(self._parameters["initial_offspring_pool_size"])
        base = last_generation[["genotype", "source_code", "parent_id"]].copy()
        _, offspring_by_id, _ = self._learn_and_replicate(base, pool_size, last)
        return self._select_offspring(last_generation, offspring_by_id), pool_size

    # ------------------------------------------------------------------------------------------
    def _learn_and_replicate(self, current: pd.DataFrame, pool_size: int, generation: int):
        p = self._parameters
        sources = list(current["source_code"])
        comm = self._comm
        plan = plan_generation(sources, self._cache, float(p["max_serann_parameters"]), comm)
        parts = lpt_partition(plan.costs, comm.world_size, plan.arch_keys, speeds=self._speeds.factors)
        local = [int(plan.trainable[i]) for i in parts[comm.rank]]
        # the shard is this many reference pool jobs: give the watchdog that many job timeouts
        self._watchdog.arm(f"generation {generation}", job_scale(len(local)))
        ids = list(current.index)
        genotypes = np.stack([np.asarray(g, np.float64) for g in current["genotype"]])
        position = {int(t): k for k, t in enumerate(plan.trainable)}
        t_shard = time.perf_counter()
        res = self._worker.run(local, [ids[i] for i in local], genotypes[local] if local else genotypes[:0],
                               [plan.results[i].ir for i in local], int(pool_size), generation,
                               self._random_seed, positions=[position[i] for i in local],
                               n_trainable=len(plan.trainable))
        t_shard = time.perf_counter() - t_shard
        # one packed all-gather: host header (indices, metrics, timings, GPU index) + the offspring bits,
        # which stay on the device from the replication epilogue to the collective (RCCL)
        head = pack_header(res.indices, res.metrics, int(pool_size), int(p["genotype_size"]), res.learning_time,
                           res.replication_time, device=comm.device_index(), shard_s=t_shard)
        t_ag = time.perf_counter()
        gathered = comm.allgather_payload(head, res.packed)
        t_ag = time.perf_counter() - t_ag

        n = len(current)
        metrics = np.full((n, 4), np.nan)
        offspring_rows: Dict[int, np.ndarray] = {}
        times = {"learning_times": [], "replication_times": [], "train_flops": self._train_flops(plan)}
        measured = []
        for blob in gathered:                        # rank order
            idx, m, off, lt, rt = unpack_results(blob)
            measured.append(float(lt) if len(idx) else 0.0)
            if len(idx):
                metrics[idx] = m
                for k, i in enumerate(idx):
                    offspring_rows[int(i)] = off[k]
                times["learning_times"].append(lt)
                times["replication_times"].append(rt)
        # the cost model prices one training step (cost_model.organism_time): x steps per generation, so that
        # predicted_s and measured_s (a shard's learning seconds) are in the same unit
        spg = getattr(self._worker, "steps_per_generation", None)
        spg = spg() if callable(spg) else 0
        predicted = [float(sum(plan.costs[j] for j in part)) * max(spg, 1) for part in parts]
        times["rank_predicted_s"], times["rank_measured_s"] = predicted, measured
        times["rank_factors"] = self._speeds.update(predicted, measured)
        # per-rank load balance and the collective's own cost, for the multi-GPU records (SCALE runs): every
        # rank's GPU, organisms, predicted (cost model) and measured (learning) seconds and shard wall time
        ranks = []
        for r, blob in enumerate(gathered):
            h = unpack_header(blob)
            ranks.append(dict(rank=r, device=h["device"], organisms=h["organisms"],
                              predicted_s=round(predicted[r], 4), measured_s=round(h["learning_s"], 4),
                              shard_s=round(h["shard_s"], 4)))
        times["ranks"] = ranks
        times["allgather_s"] = t_ag
        times["allgather_bytes"] = int(sum(len(b) for b in gathered))

        models_info = pd.DataFrame(index=current.index)
        models_info["parameters_count"] = [r.parameters_count for r in plan.results]
        models_info["loss_balance"] = [r.loss_balance for r in plan.results]
        models_info["is_valid"] = plan.is_valid
        models_info["is_overweight"] = plan.is_overweight
        models_info["classification_validation_accuracy"] = metrics[:, 0]
        models_info["classification_training_accuracy"] = metrics[:, 1]
        models_info["classification_test_accuracy"] = metrics[:, 2]
        models_info["replication_mse"] = metrics[:, 3]
        # deterministic table order (the reference uses job-completion order)
        offspring_by_id = {ids[i]: offspring_rows[i].astype(np.float64) for i in sorted(offspring_rows)}
        return models_info, offspring_by_id, times

    def _train_flops(self, plan) -> float:
        """Model FLOPs of this generation's training (forward + backward = 3x the forward FLOPs per
        sample, over every training row of every epoch, summed over the trainable organisms): the
        work measure that makes generations with different evolved populations comparable."""
        cfg = getattr(self._worker, "cfg", None)
        data = getattr(self._worker, "data", None)
        if cfg is None or data is None:
            return float("nan")
        rows = cfg.split(len(data.train_x)) * int(cfg.epochs)
        return float(sum(3.0 * plan.results[i].ir.flops_per_sample() for i in plan.trainable) * rows)

    # ------------------------------------------------------------------------------------------
    def _select_offspring(self, current: pd.DataFrame, offspring_by_id: Dict[str, np.ndarray]) -> pd.DataFrame:
        strategy = {"random": self._random_offspring_selection,
                    "best": self._best_offspring_selection}.get(self._parameters["offspring_selection_strategy"])
        if strategy is None:
            raise ValueError("Unknown offspring selection strategy")
        offspring_ids, parent_ids, genotypes = [], [], []
        # column dicts: per-cell DataFrame.at lookups cost ~10 us each (thousands per generation at pop 1000)
        geno_of = dict(zip(current.index, current["genotype"].values))
        num_of = dict(zip(current.index, current["num_offspring"].values))
        for parent_id, pool in offspring_by_id.items():
            parent_genotype = np.asarray(geno_of[parent_id], dtype=np.float64)
            num = int(num_of[parent_id])
            pool = np.round(np.clip(pool, 0, 1))
            selected = strategy(parent_genotype, num, pool)
            selected = self._probabilistic_proofreading(parent_genotype, selected)
            offspring_ids += self._new_ids(num)
            parent_ids += [parent_id] * num
            genotypes += list(selected)
        source_code = self._codec.decode_to_string(np.stack(genotypes)) if genotypes else []
        nxt = pd.DataFrame({"genotype": genotypes, "parent_id": parent_ids, "source_code": source_code},
                           index=pd.Index(offspring_ids, name="id"))
        if not genotypes:
            for c in ("genotype_euclidean_distance_from_parent", "genotype_hamming_distance_from_parent",
                      "source_code_levenshtein_distance_from_parent"):
                nxt[c] = []
            return nxt
        off = np.stack(genotypes)
        par = np.stack([np.asarray(geno_of[i], np.float64) for i in parent_ids])
        nxt["genotype_euclidean_distance_from_parent"] = np.sqrt(np.sum((off - par) ** 2, axis=1))
        nxt["genotype_hamming_distance_from_parent"] = (par != off).sum(axis=1) / self._parameters["genotype_size"]
        if self._comm.is_root:
            src_of = dict(zip(current.index, current["source_code"].values))
            parent_src = [src_of[i] for i in parent_ids]
            nxt["source_code_levenshtein_distance_from_parent"] = levenshtein_batch(list(source_code), parent_src)
        else:
            nxt["source_code_levenshtein_distance_from_parent"] = np.nan   # only rank 0 writes the DB
        return nxt

    def _random_offspring_selection(self, _, num, pool):
        perm = self._rng.permutation(len(pool))
        if num <= len(pool) or self._strict:
            return pool[perm[:num]]
        extra = self._rng.randint(0, len(pool), num - len(pool))
        return pool[np.concatenate([perm, extra])]

    def _best_offspring_selection(self, parent, num, pool):
        order = np.argsort(hamming(parent, pool), kind="stable")
        if num > len(pool) and not self._strict:
            order = np.concatenate([order, np.repeat(order[:1], num - len(pool))])
        return pool[order[:num]]

    def _probabilistic_proofreading(self, parent, offspring):
        ec = float(self._parameters["error_correction_probability"])
        offspring = offspring.copy()
        rows, cols = np.where(offspring != parent)
        fixed = self._rng.permutation(len(rows))[:int(ec * len(rows))]
        rows, cols = rows[fixed], cols[fixed]
        offspring[rows, cols] = parent[cols]
        return offspring

    # ------------------------------------------------------------------------------------------
    def _generation_statistics(self, info: pd.DataFrame, generation: int, times, start_time) -> dict:
        survived = info["is_valid"] & ~info["is_overweight"].astype(bool)
        g = {
            "experiment_id": self._id,
            "generation": generation,
            "start_time": start_time,
            "survival_rate": survived.mean(),
            "overweight_rate": info["is_overweight"].astype(float).mean(),
            "invalid_rate": 1 - info["is_valid"].astype(float).mean(),
            "mean_parameters_count": info["parameters_count"].mean(),
            "mean_absolute_fertility": info["absolute_fertility"].mean(),
            "absolute_fertility_std": info["absolute_fertility"].std(),
            "mean_loss_balance": info["loss_balance"].mean(),
            "mean_classification_validation_accuracy": info["classification_validation_accuracy"].mean(),
            "mean_classification_training_accuracy": info["classification_training_accuracy"].mean(),
            "mean_classification_test_accuracy": info["classification_test_accuracy"].mean(),
            "max_classification_test_accuracy": info["classification_test_accuracy"].max(),
            "mean_replication_mse": info["replication_mse"].mean(),
            "learning_time_seconds": float(np.mean(times["learning_times"])) if times["learning_times"] else np.nan,
            "replication_time_seconds": float(np.mean(times["replication_times"])) if times["replication_times"] else np.nan,
            "total_time_seconds": (datetime.now() - start_time).total_seconds(),
            "mean_classification_layers": info["classification_layers"].mean(),
            "mean_replication_layers": info["replication_layers"].mean(),
            "mean_merged_layers": info["merged_layers"].mean(),
        }
        if self._comm.is_root:
            gen = np.stack([np.asarray(x, np.float64) for x in info["genotype"]])
            gs = genotype_stats(gen, info["genotype_euclidean_distance_from_parent"].to_numpy(float),
                                info["genotype_hamming_distance_from_parent"].to_numpy(float))
            ss = source_code_stats(list(info["source_code"]),
                                   info["source_code_levenshtein_distance_from_parent"].to_numpy(float))
            g.update({f"genotype_{k}": v for k, v in gs.items()})
            g.update({f"source_code_{k}": v for k, v in ss.items()})
        return g
