"""Evaluation subsystem on CPU: samplers, SerannEvaluator (E replicas, R replications),
SampleDeepEvaluator resume + pickle output, analysis loaders over the experiment DB."""
import os
import pickle

import numpy as np
import pandas as pd
import pytest

from serann.analysis.results import (evaluations_from_pickle, genotype_to_hex, load_experiment_results,
                                     prepare_muller_plot_data)
from serann.config import default_parameters
from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
from serann.engine.base import TrainConfig
from serann.evaluation.driver import SAMPLERS, SampleDeepEvaluator
from serann.evaluation.evaluator import SerannEvaluationWorker, probabilistic_proofreading
from serann.experiment.experiment import Experiment
from serann.experiment.worker import ShardWorker
from serann.genome.codec import TableCodec
from serann.utils.db import ExperimentDB


@pytest.fixture(scope="module")
def experiment(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("ev")
    enc = synthetic_encodings()
    data = get_serann_data(enc, synthetic_mnist(n_train=800, n_test=200), n_train=800, n_test=200)
    p = default_parameters("example")
    p.update(num_seranns=5, num_generations=3, training_epochs=1)
    codec = TableCodec.from_generator(64, seed=1, ancestor=p["ancestor_genotype"])
    w = ShardWorker(p, data, "torch", "cpu", TrainConfig(epochs=1, batch_size=200))
    db = ExperimentDB(tmp / "exp.sqlite")
    Experiment("exp", enc, w, db, p, codec, random_seed=2, verbose=False).execute()
    df = load_experiment_results("exp_test_" + os.path.basename(str(tmp)), db_path=db.db_path, cache_invalidate=True)
    return df, data, codec, p, tmp


def test_results_loader_columns(experiment):
    df, *_ = experiment
    for c in ("genotype_hex", "is_mutant", "descendants", "parent_genotype_hex", "parent_generation"):
        assert c in df.columns
    assert (df[df["generation"] == 0]["parent_id"] == "experiment_ancestor_id").all()
    assert genotype_to_hex([1, 0, 1]) == "0x5"


@pytest.mark.parametrize("name", sorted(SAMPLERS))
def test_samplers(experiment, name):
    df, *_ = experiment
    params = {"total_samples": 4, "generation_step": 1, "samples_per_generation": 1}
    idx = SAMPLERS[name](seed=0).sample(df, params)
    assert set(idx) <= set(df.index)


def test_proofreading_reverts_fraction():
    rng = np.random.RandomState(0)
    parent = np.zeros(100)
    off = np.ones((3, 100))
    fixed = probabilistic_proofreading(parent, off, 0.5, rng)
    assert (fixed != parent).sum() == 150
    assert (probabilistic_proofreading(parent, off, 0.0, rng) == off).all()


def test_evaluator_and_driver_resume(experiment, tmp_path):
    df, data, codec, p, _ = experiment
    ep = {k: p[k] for k in ("genotype_size", "error_correction_probability", "classification_image_dimensions",
                            "num_classification_classes", "training_epochs", "training_batch_size")}
    worker = SerannEvaluationWorker(ep, data, codec, num_evaluations=2, replications_per_evaluation=4, engine="torch",
                                    device="cpu", train_cfg=TrainConfig(epochs=1, batch_size=200))
    ids = list(df.index[:4])
    out = tmp_path / "ev.pkl"
    ev = SampleDeepEvaluator(df, str(out), ids, worker, batch=2, log=lambda *a, **k: None)
    res = ev.run()
    assert set(res) == set(ids)
    valid = [i for i in ids if df.at[i, "is_valid"] and not df.at[i, "is_overweight"]]
    for i in valid:
        r = res[i]
        assert len(r["classification_accuracy"]) == 2
        assert len(r["mutation_rate"]) == 2 and sum(r["mutation_rate"][0].values()) == 4
        assert sum(r["offspring_survival"][1].values()) == 4
    with open(out, "rb") as f:
        assert set(pickle.load(f)) == set(ids)
    # resume: everything already evaluated -> nothing recomputed, backup written
    ev2 = SampleDeepEvaluator(df, str(out), ids, worker, batch=2, log=lambda *a, **k: None)
    assert ev2.run() == res
    assert (tmp_path / "ev_backup.pkl").exists()
    flat = evaluations_from_pickle(str(out))
    assert set(flat["serann_id"]) == set(ids)


def test_evaluation_dies_midway_and_resumes_from_pickle(experiment, tmp_path, monkeypatch):
    """An injected death after the first pickle (SERANN_FAULT_INJECT evaluated=2): the relaunch reads the
    pickle, evaluates only what is missing, and ends with the same results as an uninterrupted run."""
    from serann.utils.faults import InjectedFault
    df, data, codec, p, _ = experiment
    ep = {k: p[k] for k in ("genotype_size", "error_correction_probability", "classification_image_dimensions",
                            "num_classification_classes", "training_epochs", "training_batch_size")}

    def worker():
        return SerannEvaluationWorker(ep, data, codec, num_evaluations=2, replications_per_evaluation=4,
                                      engine="torch", device="cpu", train_cfg=TrainConfig(epochs=1, batch_size=200))
    ids = list(df.index[:6])
    quiet = lambda *a, **k: None  # noqa: E731
    full = SampleDeepEvaluator(df, str(tmp_path / "full.pkl"), ids, worker(), batch=2, log=quiet).run()
    out = tmp_path / "cut.pkl"
    monkeypatch.setenv("SERANN_FAULT_INJECT", "evaluated=2,mode=raise")
    with pytest.raises(InjectedFault):
        SampleDeepEvaluator(df, str(out), ids, worker(), batch=2, log=quiet, save_every=2).run()
    monkeypatch.delenv("SERANN_FAULT_INJECT")
    with open(out, "rb") as f:
        saved = pickle.load(f)
    assert sum(1 for v in saved.values() if len(v)) == 2
    w = worker()
    calls = []
    orig = w.run_many
    w.run_many = lambda rows: calls.append(len(rows)) or orig(rows)
    res = SampleDeepEvaluator(df, str(out), ids, w, batch=2, log=quiet, save_every=2).run()
    assert sum(calls) == 4                      # only the missing four were evaluated
    assert res.keys() == full.keys()
    for i in ids:
        # (an organism that cannot be evaluated reports nan in both runs)
        np.testing.assert_array_equal(res[i]["classification_accuracy"], full[i]["classification_accuracy"], err_msg=i)


def test_muller_plot_data(experiment):
    df, *_ = experiment
    pops, adj = prepare_muller_plot_data(df, frequency_threshold=0.0)
    assert {"Generation", "Identity", "Population"} <= set(pops.columns)
    assert (pops.groupby("Generation")["Population"].sum() == 5).all()


def test_load_experiment_data_by_path(experiment):
    from serann.analysis.results import load_experiment_data
    df, data, codec, p, tmp = experiment
    path = str(tmp / "exp.sqlite")
    d = load_experiment_data(path, cache_invalidate=True)
    assert len(d) == len(df) and not any(c.startswith("parent_") and c not in ("parent_id", "parent_genotype_hex")
                                         for c in d.columns)
    g0 = d[d["generation"] == 0]
    assert (g0["parent_id"] == "experiment_ancestor_id").all()
    assert (g0["parent_genotype_hex"] == "experiment_ancestor_genotype_hex").all()
    assert d["genotype"].iloc[0].dtype.kind == "i" and d["descendants"].ge(0).all()
    # total descendants of generation 0 = every later organism
    assert d.loc[g0.index, "descendants"].sum() == (d["generation"] > 0).sum()
    ev = pd.DataFrame({"genotype_hex": [d["genotype_hex"].iloc[0]], "fitness": [0.5], "mutation_rate": [0.1]})
    j = load_experiment_data(path, deep_evaluations=ev)          # cached frame + evaluation join
    assert j.loc[j["genotype_hex"] == ev["genotype_hex"][0], "fitness"].eq(0.5).all()
    assert j["fitness"].isna().sum() == (j["genotype_hex"] != ev["genotype_hex"][0]).sum()


def test_replica_seeds_follow_the_genotype(experiment):
    """A genotype's replica initialisations (and so its accuracies) do not depend on its position in the
    evaluated batch: evaluating X alone or after another genotype gives the same accuracies."""
    from serann.evaluation.evaluator import SerannEvaluator
    df, data, codec, p, _ = experiment
    ep = {k: p[k] for k in ("genotype_size", "error_correction_probability", "classification_image_dimensions",
                            "num_classification_classes", "training_epochs", "training_batch_size")}
    ok = df[(df["is_valid"] == True) & (df["is_overweight"] == False)]  # noqa: E712
    hexes = ok["genotype_hex"].drop_duplicates()
    assert len(hexes) >= 1
    x = np.asarray(ok.loc[hexes.index[0], "genotype"], np.float64)
    y = 1.0 - x

    def ev():
        return SerannEvaluator(ep, data, codec, num_evaluations=2, replications_per_evaluation=2, engine="torch",
                               device="cpu", train_cfg=TrainConfig(epochs=1, batch_size=200))
    alone = ev().evaluate_many([x])[0]
    second = ev().evaluate_many([y, x])[1]
    assert alone["classification_accuracy"] == second["classification_accuracy"]
