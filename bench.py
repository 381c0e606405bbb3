#!/usr/bin/env python
"""Headline benchmark: SeRANN generations at pop = 125 x N GPUs (pop = 1000 at 8 GPUs).

BASELINE.json metric: "seconds/generation at pop=1000 (8 GPUs) + SeRANN trained/sec at 1/2/4/8 GPUs".
One *step* is one full generation of the full_experiment.json config: decode, train every organism
5 epochs x 76 steps (batch 750, Keras Adam), validation each epoch, test evaluation, replication,
fertility, multinomial offspring counts, selection + proofreading, decode, population statistics and
the SQLite writes.  Per-GPU work is fixed as N grows (125 organisms per GPU) -> weak scaling.

Data is synthetic (no network): MNIST-shaped learnable images, random genotype encodings, random-init
weights, and the synthetic table codec that decodes genotypes into architectures drawn from the
reference generator distribution.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_SERANN_PER_SEC = 0.40   # pop=50, ~126 s/generation on 1x Titan X (3.5 h / 100 gens)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pop-per-gpu", type=int, default=125)
    ap.add_argument("--engine", default="auto")
    ap.add_argument("--parameters", default=None)
    ap.add_argument("--dump-population", default=None,
                    help="write the source codes of the last generation (JSON list) for scripts/bench_step.py")
    ap.add_argument("--profile-dir", default=None,
                    help="torch.profiler Chrome trace of the run per rank (diagnostics; not a headline timing)")
    ap.add_argument("--no-fixed-pop", action="store_true",
                    help="skip the fixed-population step timings printed after the timed generations")
    args = ap.parse_args()

    import numpy as np
    import torch
    from serann.config import default_parameters, load_parameters
    from serann.experiment.experiment import Experiment
    from serann.experiment.runner import setup
    from serann.parallel.comm import make_comm
    from serann.utils.db import ExperimentDB

    comm = make_comm()
    # the driver's contract: one rank per GPU of one node.  Fail fast on a launch that does not match --gpus
    # or ranks that share / miss their GPU, instead of timing a different configuration
    if comm.world_size != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {comm.world_size}: launch one rank per GPU")
    if torch.cuda.is_available() and args.engine in ("auto", "hip"):
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.current_device() != local_rank:
            raise SystemExit(f"bench.py: rank {comm.rank} computes on cuda:{torch.cuda.current_device()}, "
                             f"not its LOCAL_RANK {local_rank}")
        if torch.cuda.device_count() < args.gpus and comm.world_size > 1:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but only {torch.cuda.device_count()} visible GPUs")
    params = load_parameters(args.parameters) if args.parameters else default_parameters("full_experiment")
    pop = args.pop_per_gpu * comm.world_size
    params["num_seranns"] = pop
    params["num_generations"] = args.warmup + args.steps
    s = setup(params, engine=args.engine, comm=comm)
    is_cuda = s.device.startswith("cuda")

    db = None
    tmpdir = tempfile.mkdtemp(prefix="serann_bench_")
    if comm.is_root:
        db = ExperimentDB(os.path.join(tmpdir, f"{uuid.uuid4()}.sqlite"))
    exp = Experiment("bench", s.encodings, s.worker, db, params, s.codec, comm=comm, random_seed=79375,
                     verbose=bool(os.environ.get("SERANN_VERBOSE")))

    marks = {}

    def on_generation(gen, rec):
        if gen == args.warmup - 1:
            if is_cuda:
                torch.cuda.synchronize()
            comm.barrier()
            marks["t0"] = time.perf_counter()
        if comm.is_root:
            print(json.dumps({"progress": rec}), file=sys.stderr, flush=True)

    if args.warmup == 0:
        comm.barrier()
        marks["t0"] = time.perf_counter()
    from serann.utils.trace import profiled
    with profiled(args.profile_dir, f"rank{comm.rank}"):
        hist = exp.execute(on_generation=on_generation)
    if is_cuda:
        torch.cuda.synchronize()
    comm.barrier()
    t1 = time.perf_counter()
    timed = [h for h in hist if h["generation"] >= args.warmup]
    k = len(timed)
    elapsed = t1 - marks.get("t0", t1)
    elapsed = comm.allreduce_max(elapsed)
    # Fixed-population step times (after the timed region, rank 0 only): the evolved trajectory -- and with it the
    # work of a generation -- moves with every rounding or data change, so kernel progress across trees is read
    # from two fixed populations instead: ms per captured-graph training step at 4 stream groups, batch 750
    fixed = None
    if comm.is_root and is_cuda and s.engine == "hip" and not args.no_fixed_pop:
        fixed = fixed_population_ms(s.data)
    comm.barrier()
    if comm.is_root:
        sec_per_gen = elapsed / max(k, 1)
        value = pop * k / elapsed if elapsed > 0 and k else 0.0
        out = {
            "metric": "serann_trained_per_sec",
            "value": value,
            "unit": "SeRANN/s (population organisms processed per second, whole job)",
            "n_gpus": comm.world_size,
            "steps": k,
            "warmup": args.warmup,
            "ms_per_step": sec_per_gen * 1000.0,
            "seconds_per_generation": sec_per_gen,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": value / BASELINE_SERANN_PER_SEC,
            "dtype": "bf16",
            "data": "synthetic (MNIST-shaped images, random genotype encodings, table codec over "
                    "generator-sampled architectures, random-init weights)",
            "engine": s.engine,
            "config": {"model": "SeRANN population, full_experiment.json (5 epochs, batch 750, "
                                "architectures from the reference generator distribution)",
                       "global_batch": int(params["training_batch_size"]), "seq_len": int(params["genotype_size"]),
                       "population": pop, "parallelism": f"population-sharded dp{comm.world_size}"},
            # per generation: "ranks" (GPU index, organisms, predicted / measured learning seconds and shard
            # wall time of every rank), "allgather_s" / "allgather_bytes" (the one collective per generation)
            "generations": timed,
            # work normalisation: the evolved population (and so the work of a generation) depends on the
            # seeded trajectory; model FLOPs of training per generation and the rate achieved on them
            "train_tflop_per_generation": float(np.mean([h.get("train_tflop", float("nan")) for h in timed]))
            if timed else None,
            "achieved_model_tflops": (sum(h.get("train_tflop", 0.0) for h in timed) / elapsed)
            if elapsed > 0 and timed else None,        # (train_tflop counts the whole population)
            # trajectory-independent kernel progress: populations/*.json, 4 stream groups, graph replay (not timed
            # above; measured after the K generations)
            "fixed_pop_ms_per_step": fixed,
        }
        print(json.dumps(out), flush=True)
    if comm.is_root and args.dump_population and db is not None:
        import sqlite3
        con = sqlite3.connect(db.db_path)
        rows = con.execute("select source_code from serann where generation = (select max(generation) from serann)"
                           " and is_valid = 1 and is_overweight = 0").fetchall()
        with open(args.dump_population, "w") as f:
            json.dump([r[0] for r in rows], f)
    comm.shutdown()


def fixed_population_ms(data, streams: int = 4, steps: int = 60) -> dict:
    """ms per replayed training step (batch 750, ``streams`` stream groups) of the two fixed populations in
    populations/: the generation-3 mix of the bench trajectory (106 organisms) and 125 clones of the example.json
    ancestor (scripts/bench_step.py measures the same)."""
    import torch
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.genome.interpreter import try_interpret
    out = {}
    root = os.path.dirname(os.path.abspath(__file__))
    saved = os.environ.get("SERANN_STREAMS")
    os.environ["SERANN_STREAMS"] = str(streams)
    try:
        for name in ("bench_gen3_pop125", "ancestor_pop125"):
            with open(os.path.join(root, "populations", f"{name}.json")) as f:
                irs = [try_interpret(src).ir for src in json.load(f)][:125]
            cfg = TrainConfig(epochs=1, batch_size=750, val_every_epoch=False, max_steps_per_epoch=steps)
            eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
            eng.fit(data, cfg)
            torch.cuda.synchronize()
            out[name] = round(float(eng.timings.get("replay_ms_per_step", float("nan"))), 3)
            eng.close()
            del eng
    finally:
        if saved is None:
            os.environ.pop("SERANN_STREAMS", None)
        else:
            os.environ["SERANN_STREAMS"] = saved
    out["streams"] = streams
    return out


if __name__ == "__main__":
    main()
