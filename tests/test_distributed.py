"""Multi-process SPMD on CPU (gloo, world_size 2 and 4): the sharded run must write exactly the same
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


def _worker(rank, world, port, db_path):
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
    Experiment("dist", enc, w, db, p, codec, comm=comm, random_seed=3, verbose=False).execute()
    comm.shutdown()


def _read(path):
    con = sqlite3.connect(path)
    cols = ("id, generation, genotype, source_code, parent_id, num_offspring, is_valid, "
            "classification_validation_accuracy, replication_mse")
    return pd.read_sql(f"select {cols} from serann order by generation, id", con)


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_world_matches_world1(tmp_path, world):
    p1 = str(tmp_path / "w1.sqlite")
    _worker(0, 1, _free_port(), p1)
    p2 = str(tmp_path / f"w{world}.sqlite")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, p2)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(300)
        assert pr.exitcode == 0
    a, b = _read(p1), _read(p2)
    pd.testing.assert_frame_equal(a, b, check_exact=False, rtol=1e-5, atol=1e-6)
