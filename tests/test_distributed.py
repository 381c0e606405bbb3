"""Multi-process SPMD on CPU (gloo, world_size 2, 4 and 8 -- the production rank count): the sharded run must write exactly the same
experiment DB as the single-process run (partition-independent organism seeds, shared batch
permutation, replicated control plane, one packed all-gather per generation)."""
import os
import socket
import sqlite3

import pandas as pd
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, db_path, perf_log=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    torch.set_num_threads(1)
    from serann.config import default_parameters
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.experiment.experiment import Experiment
    from serann.experiment.worker import ShardWorker
    from serann.genome.codec import TableCodec
    from serann.parallel.comm import LocalComm, TorchDistComm
    from serann.utils.db import ExperimentDB

    comm = TorchDistComm(backend="gloo") if world > 1 else LocalComm()
    enc = synthetic_encodings()
    data = get_serann_data(enc, synthetic_mnist(n_train=1000, n_test=200), n_train=1000, n_test=200)
    p = default_parameters("example")
    p.update(num_seranns=6, num_generations=2, training_epochs=1)
    codec = TableCodec.from_generator(128, seed=1, ancestor=p["ancestor_genotype"])
    w = ShardWorker(p, data, "torch", "cpu", TrainConfig(epochs=1, batch_size=250))
    db = ExperimentDB(db_path) if comm.is_root else None
    Experiment("dist", enc, w, db, p, codec, comm=comm, random_seed=3, verbose=False,
               perf_log=perf_log if comm.is_root else None).execute()
    comm.shutdown()


def _read(path):
    con = sqlite3.connect(path)
    cols = ("id, generation, genotype, source_code, parent_id, num_offspring, is_valid, "
            "classification_validation_accuracy, replication_mse")
    return pd.read_sql(f"select {cols} from serann order by generation, id", con)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_world_matches_world1(tmp_path, world):
    p1 = str(tmp_path / "w1.sqlite")
    _worker(0, 1, _free_port(), p1)
    p2 = str(tmp_path / f"w{world}.sqlite")
    log = str(tmp_path / f"w{world}.jsonl")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, p2, log)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(300)
        assert pr.exitcode == 0
    a, b = _read(p1), _read(p2)
    pd.testing.assert_frame_equal(a, b, check_exact=False, rtol=1e-5, atol=1e-6)
    # the per-generation records explain a multi-GPU run: every rank's device, organisms, predicted and
    # measured seconds and shard wall time, and the cost of the one collective (bench.py prints these)
    import json
    recs = [json.loads(line) for line in open(log)]
    assert len(recs) == 2
    for rec in recs:
        ranks = rec["ranks"]
        assert [r["rank"] for r in ranks] == list(range(world))
        assert all(r["device"] == -1 for r in ranks)                     # gloo / CPU ranks
        assert sum(r["organisms"] for r in ranks) == rec["valid"]
        assert all(r["shard_s"] >= r["measured_s"] >= 0 and r["predicted_s"] >= 0 for r in ranks)
        assert rec["allgather_s"] > 0 and rec["allgather_bytes"] > 0
        assert rec["rank_imbalance"] >= 1.0 and len(rec["rank_factors"]) == world
    # predicted_s is in the unit of measured_s (learning seconds of the generation): the cost model's seconds per
    # step of every trained organism times the generation's steps (1 epoch x ceil(950 / 250))
    from serann.experiment.cost_model import organism_time
    from serann.genome.interpreter import interpret
    con = sqlite3.connect(p2)
    for rec in recs:
        rows = con.execute("select source_code from serann where generation = ? and is_valid = 1 and "
                           "is_overweight = 0", (rec["generation"],)).fetchall()
        want = 4 * sum(organism_time(interpret(r[0])) for r in rows)
        got = sum(r["predicted_s"] for r in rec["ranks"])
        assert abs(got - want) <= 1e-3 * want + 1e-4 * world, (got, want)


def test_rank_speed_model_balances_injected_slowdowns():
    """Per-rank slowdowns the cost model cannot see (a power-capped or shared GPU): after 3 generations of
    online correction the true shard times are within 3 % of their mean (max / mean <= 1.03), on fresh
    heavy-tailed populations every generation, with 2 % timing noise."""
    import numpy as np
    from serann.parallel.partition import RankSpeedModel, lpt_partition
    rng = np.random.default_rng(0)
    slow = np.array([1.0, 1.6, 1.0, 0.7, 1.25, 1.0, 1.0, 0.9])
    world = len(slow)
    model = RankSpeedModel(world)
    ratios = []
    for gen in range(4):
        costs = rng.lognormal(0.0, 1.0, 1000)                   # p99 / median ~ 10
        parts = lpt_partition(costs, world, speeds=model.factors)
        pred = np.array([costs[p].sum() for p in parts])
        true = pred * slow * 0.37                               # unknown global scale as well
        ratios.append(true.max() / true.mean())
        model.update(pred, true * rng.normal(1.0, 0.02, world))
    assert ratios[0] > 1.2                                      # the uncorrected split is badly skewed
    assert ratios[3] <= 1.03, ratios
    f = np.array(model.factors)
    assert np.allclose(f / np.exp(np.log(f).mean()), slow / np.exp(np.log(slow).mean()), rtol=0.05)


def test_speed_aware_lpt_is_plain_lpt_at_unit_speeds():
    from serann.parallel.partition import lpt_partition
    costs = [5, 3, 3, 2, 2, 2, 1]
    assert lpt_partition(costs, 3) == lpt_partition(costs, 3, speeds=[1.0, 1.0, 1.0])
    # a 2x slower rank gets about a third of the work of each fast one
    parts = lpt_partition([1.0] * 30, 3, speeds=[1.0, 2.0, 1.0])
    assert sorted(len(p) for p in parts) == [6, 12, 12]
