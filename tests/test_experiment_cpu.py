"""End-to-end generation loop on the CPU torch oracle (BASELINE config #1: pop=2, 1 generation),
SQLite schema parity with the reference writer, and determinism / resume."""
import sqlite3

import numpy as np
import pandas as pd
import pytest

from serann.config import default_parameters
from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
from serann.engine.base import TrainConfig
from serann.experiment.experiment import Experiment
from serann.experiment.worker import ShardWorker
from serann.genome.codec import TableCodec
from serann.utils.db import ExperimentDB

SERANN_COLUMNS = ["id", "genotype", "source_code", "parent_id", "genotype_euclidean_distance_from_parent",
                  "genotype_hamming_distance_from_parent", "source_code_levenshtein_distance_from_parent",
                  "experiment_id", "generation", "num_offspring", "parameters_count", "loss_balance", "is_valid",
                  "is_overweight", "classification_validation_accuracy", "classification_training_accuracy",
                  "classification_test_accuracy", "replication_mse", "absolute_fertility", "relative_fertility",
                  "classification_layers", "replication_layers", "merged_layers"]
GEN_COLUMNS = ["experiment_id", "generation", "start_time", "survival_rate", "overweight_rate", "invalid_rate",
               "mean_parameters_count", "mean_absolute_fertility", "absolute_fertility_std", "mean_loss_balance",
               "mean_classification_validation_accuracy", "mean_classification_training_accuracy",
               "mean_classification_test_accuracy", "max_classification_test_accuracy", "mean_replication_mse",
               "learning_time_seconds", "replication_time_seconds", "total_time_seconds",
               "mean_classification_layers", "mean_replication_layers", "mean_merged_layers",
               "genotype_mean_pairwise_euclidean_distance", "genotype_mean_pairwise_hamming_distance",
               "genotype_mean_euclidean_distance_from_parent", "genotype_mean_hamming_distance_from_parent",
               "genotype_shannon_index", "genotype_nucleotide_diversity", "genotype_species_richness",
               "source_code_median_levenshtein_distance_from_parent", "source_code_shannon_index",
               "source_code_species_richness"]


@pytest.fixture(scope="module")
def small_data():
    enc = synthetic_encodings()
    return enc, get_serann_data(enc, synthetic_mnist(n_train=1200, n_test=300), n_train=1200, n_test=300)


def _run(tmp_path, small_data, pop=2, gens=1, seed=5, name="e.sqlite"):
    enc, data = small_data
    p = default_parameters("example")
    p.update(num_seranns=pop, num_generations=gens, training_epochs=1)
    codec = TableCodec.from_generator(128, seed=1, ancestor=p["ancestor_genotype"])
    w = ShardWorker(p, data, "torch", "cpu", TrainConfig(epochs=1, batch_size=200))
    db = ExperimentDB(tmp_path / name)
    e = Experiment("exp", enc, w, db, p, codec, random_seed=seed, verbose=False)
    hist = e.execute()
    return db, hist


def test_pop2_one_generation_schema(tmp_path, small_data):
    db, hist = _run(tmp_path, small_data)
    con = sqlite3.connect(db.db_path)
    serann = pd.read_sql("select * from serann", con)
    gens = pd.read_sql("select * from generations", con)
    info = pd.read_sql("select * from execution_info", con)
    assert list(serann.columns) == SERANN_COLUMNS
    assert list(gens.columns) == GEN_COLUMNS
    assert len(serann) == 2 and len(gens) == 1 and len(info) == 1
    assert serann["is_valid"].all()
    assert serann["num_offspring"].sum() == 2
    assert np.isclose(serann["relative_fertility"].sum(), 1.0)
    assert serann["genotype"].iloc[0].startswith("[0, 0, 0")
    assert info["ancestor_genotype"].iloc[0].startswith("0000000111")


def test_multi_generation_determinism(tmp_path, small_data):
    db1, h1 = _run(tmp_path, small_data, pop=4, gens=3, name="a.sqlite")
    db2, h2 = _run(tmp_path, small_data, pop=4, gens=3, name="b.sqlite")
    a = pd.read_sql("select id, genotype, source_code, num_offspring from serann", sqlite3.connect(db1.db_path))
    b = pd.read_sql("select id, genotype, source_code, num_offspring from serann", sqlite3.connect(db2.db_path))
    pd.testing.assert_frame_equal(a, b)
    later = pd.read_sql("select * from serann where generation > 0", sqlite3.connect(db1.db_path))
    assert later["parent_id"].notna().all()
    assert later["genotype"].iloc[0].startswith("[0.0") or later["genotype"].iloc[0].startswith("[1.0")


def test_injected_fault_then_exact_resume(tmp_path, small_data, monkeypatch):
    """a rank dies at generation 2 (SERANN_FAULT_INJECT); relaunching from the DB
    (start generation = rows in ``generations``, as ``--resume-experiment-id`` does) continues from
    ``resume_state`` and writes exactly the rows of an uninterrupted run."""
    from serann.utils.faults import InjectedFault
    ref_db, _ = _run(tmp_path, small_data, pop=4, gens=4, name="ref.sqlite")

    enc, data = small_data
    p = default_parameters("example")
    p.update(num_seranns=4, num_generations=4, training_epochs=1)
    codec = TableCodec.from_generator(128, seed=1, ancestor=p["ancestor_genotype"])

    def experiment(db, start):
        w = ShardWorker(p, data, "torch", "cpu", TrainConfig(epochs=1, batch_size=200))
        return Experiment("exp", enc, w, db, p, codec, random_seed=5, verbose=False, start_generation=start)

    db = ExperimentDB(tmp_path / "crash.sqlite")
    monkeypatch.setenv("SERANN_FAULT_INJECT", "generation=2")
    with pytest.raises(InjectedFault):
        experiment(db, 0).execute()
    assert db.get_generations_count() == 2
    monkeypatch.delenv("SERANN_FAULT_INJECT")
    hist = experiment(db, db.get_generations_count()).execute()
    assert [h["generation"] for h in hist] == [2, 3]
    assert set(hist[0]["phases"]) >= {"learn_and_replicate", "statistics", "db_write", "selection"}

    cols = ("id, genotype, source_code, parent_id, generation, num_offspring, classification_validation_accuracy,"
            " replication_mse")
    a = pd.read_sql(f"select {cols} from serann", sqlite3.connect(ref_db.db_path))
    b = pd.read_sql(f"select {cols} from serann", sqlite3.connect(db.db_path))
    pd.testing.assert_frame_equal(a, b)
    info = pd.read_sql("select * from execution_info", sqlite3.connect(db.db_path))
    assert len(info) == 2                                  # one execution_info row per launch


def test_fault_spec_parsing():
    from serann.utils.faults import InjectedFault, maybe_inject, parse
    assert parse("generation=3,rank=1,mode=exit") == {"generation": 3, "evaluated": None, "rank": 1, "mode": "exit"}
    assert parse("evaluated=100,mode=exit") == {"generation": None, "evaluated": 100, "rank": None, "mode": "exit"}
    assert parse("") is None
    with pytest.raises(ValueError):
        parse("rank=1")
    with pytest.raises(ValueError):
        parse("generation=1,evaluated=2")                  # exactly one trigger
    maybe_inject(3, rank=0, spec="generation=3,rank=1")     # other rank: no fault
    maybe_inject(2, rank=1, spec="generation=3,rank=1")     # other generation: no fault
    with pytest.raises(InjectedFault):
        maybe_inject(3, rank=1, spec="generation=3,rank=1")


def test_cli_resume_keeps_started_seed(tmp_path, monkeypatch):
    """A run started with ``-s N``, killed, and resumed with ``-r <id>`` alone must continue with seed N
    (organism weight-init and epoch-permutation seeds derive from it): same rows as an uninterrupted run."""
    import json

    from serann.cli import run_experiment as cli
    from serann.config import experiment_config
    from serann.utils.faults import InjectedFault
    monkeypatch.setitem(experiment_config, "experiment_results_dir", str(tmp_path))
    p = default_parameters("example")
    p.update(num_seranns=3, num_generations=3, training_epochs=1)
    pf = tmp_path / "p.json"
    pf.write_text(json.dumps(p))
    common = ["--engine", "torch", "--codec", "table", "--data-subset", "1200"]
    ref_id = cli.main(["-p", str(pf), "-s", "4242", *common])
    monkeypatch.setenv("SERANN_FAULT_INJECT", "generation=2")
    with pytest.raises(InjectedFault):
        cli.main(["-p", str(pf), "-s", "4242", *common])
    monkeypatch.delenv("SERANN_FAULT_INJECT")
    crashed = [f.stem for f in tmp_path.glob("*.sqlite") if f.stem != ref_id]
    assert len(crashed) == 1
    cli.main(["-r", crashed[0], *common])
    cols = "id, genotype, source_code, parent_id, generation, num_offspring, classification_validation_accuracy"
    a = pd.read_sql(f"select {cols} from serann", sqlite3.connect(tmp_path / f"{ref_id}.sqlite"))
    b = pd.read_sql(f"select {cols} from serann", sqlite3.connect(tmp_path / f"{crashed[0]}.sqlite"))
    pd.testing.assert_frame_equal(a, b)
    info = pd.read_sql("select random_seed from execution_info", sqlite3.connect(tmp_path / f"{crashed[0]}.sqlite"))
    assert [int(s) for s in info["random_seed"]] == [4242, 4242]


def test_resume_state_is_plain_data(tmp_path):
    """The resume state round-trips through JSON + npz (no pickle), NaN genotypes included."""
    db = ExperimentDB(tmp_path / "r.sqlite")
    df = pd.DataFrame({"genotype": [np.array([0.0, 1.0, np.nan]), np.array([1.0, 1.0, 0.0])],
                       "source_code": ["a=1", "b=2"], "parent_id": [None, "p1"],
                       "genotype_hamming_distance_from_parent": [np.nan, 2.0]},
                      index=pd.Index(["i0", "i1"], name="id"))
    rng = np.random.RandomState(3)
    rng.normal()
    db.save_resume_state(4, {"next_generation": df, "pool_size": 7, "rng": rng.get_state(), "random_seed": 99})
    st = db.get_resume_state(4)
    assert st["pool_size"] == 7 and st["random_seed"] == 99
    got = st["next_generation"]
    assert list(got.index) == ["i0", "i1"] and list(got.columns) == list(df.columns)
    assert np.array_equal(got["genotype"].iloc[0], df["genotype"].iloc[0], equal_nan=True)
    assert got["parent_id"].iloc[0] is None and got["parent_id"].iloc[1] == "p1"
    r2 = np.random.RandomState()
    r2.set_state(st["rng"])
    assert r2.normal() == rng.normal()
    blob = sqlite3.connect(db.db_path).execute("select arrays from resume_state").fetchone()[0]
    assert blob[:2] == b"PK"                                  # an npz archive


def test_replication_bits_non_finite():
    from serann.experiment.worker import replication_bits
    o = np.array([[0.2, 0.7, np.nan, np.inf, -np.inf, 1.5, -0.3]])
    assert replication_bits(o).tolist() == [[0, 1, 0, 1, 0, 1, 0]]
