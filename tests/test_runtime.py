"""Population statistics, native Levenshtein, SQLite schema, fertility, partitioning, packing."""
import numpy as np
import pandas as pd
from scipy.spatial.distance import cdist, pdist

from serann.parallel.comm import pack_results, unpack_results
from serann.parallel.partition import lpt_partition
from serann.utils.db import ExperimentDB
from serann.utils.levenshtein import _py_levenshtein, levenshtein, levenshtein_batch
from serann.utils.stats import fertility, genotype_stats, source_code_stats


def ref_hamming(a, b, *args, **kwargs):
    return np.not_equal(a, b).sum(axis=-1) / np.shape(a)[-1]


def test_genotype_stats_match_scipy_definitions():
    rng = np.random.default_rng(0)
    g = rng.integers(0, 2, (40, 100)).astype(float)
    g[5] = g[3]
    s = genotype_stats(g, np.full(40, np.nan), np.full(40, np.nan))
    assert np.isclose(s["mean_pairwise_euclidean_distance"], np.mean(pdist(g)))
    assert np.isclose(s["mean_pairwise_hamming_distance"], np.mean(pdist(g, metric=ref_hamming)))
    assert np.isclose(s["nucleotide_diversity"], cdist(g, g, metric=ref_hamming).sum())
    dist = pd.Series([str(x) for x in g]).value_counts(normalize=True)
    assert np.isclose(s["shannon_index"], -np.sum(dist * np.log(dist)))
    assert s["species_richness"] == 39


def test_source_code_stats():
    s = source_code_stats(["a", "a", "b"], [1.0, np.nan, 3.0])
    assert s["species_richness"] == 2 and s["median_levenshtein_distance_from_parent"] == 2.0


def test_levenshtein_native_matches_dp():
    rng = np.random.default_rng(1)
    alpha = list("X_layer=Conv2D(,)\n")
    a = ["".join(rng.choice(alpha, rng.integers(0, 300))) for _ in range(40)]
    b = [x[: len(x) // 2] + "".join(rng.choice(alpha, 20)) for x in a]
    got = levenshtein_batch(a, b)
    assert got == [_py_levenshtein(x, y) for x, y in zip(a, b)]
    assert levenshtein("kitten", "sitting") == 3


def test_fertility_nan_handling():
    a, r = fertility(np.array([0.5, np.nan, 0.25]), 2)
    assert np.isnan(a[1]) and np.isclose(r.sum(), 1) and r[1] == 0
    a, r = fertility(np.array([np.nan, np.nan]), 1)
    assert r.sum() == 0


def test_lpt_partition_balanced_and_deterministic():
    rng = np.random.default_rng(0)
    costs = rng.lognormal(0, 1.5, 500)
    parts = lpt_partition(costs, 8)
    assert sorted(sum(parts, [])) == list(range(500))
    loads = [costs[p].sum() for p in parts]
    assert max(loads) / (sum(loads) / 8) < 1.1
    assert parts == lpt_partition(costs, 8)


def test_result_packing_roundtrip():
    idx = np.array([3, 9], np.int32)
    m = np.random.rand(2, 4)
    off = np.random.randint(0, 2, (2, 7, 100)).astype(np.uint8)
    i2, m2, o2, lt, rt = unpack_results(pack_results(idx, m, off, 1.5, 2.5))
    assert (i2 == idx).all() and np.allclose(m2, m) and (o2 == off).all() and lt == 1.5 and rt == 2.5
    i3, m3, o3, _, _ = unpack_results(pack_results(np.zeros(0, np.int32), np.zeros((0, 4)), np.zeros((0, 7, 100)), 0, 0))
    assert len(i3) == 0


def test_db_roundtrip(tmp_path):
    db = ExperimentDB(tmp_path / "x.sqlite")
    params = {"num_seranns": 2, "num_generations": 3, "ancestor_genotype": [0, 1, 1],
              "classification_image_dimensions": [28, 28], "offspring_pool_size_factor": 5,
              "training_epochs": 5, "selection_pressure": 1}
    db.save_execution_info(pd.Timestamp("2020-01-01"), params)
    db.save_execution_info(pd.Timestamp("2020-01-02"), params)
    assert db.get_executions_count() == 2
    info = db.get_last_execution_info()
    assert info["ancestor_genotype"] == [0, 1, 1] and info["classification_image_dimensions"] == [28, 28]
    df = pd.DataFrame({"genotype": [np.array([0, 1]), np.array([1., 1.])], "generation": [0, 0],
                       "is_valid": [True, False], "num_offspring": [2, 0]},
                      index=pd.Index(["a", "b"], name="id"))
    db.save_seranns_info(df)
    back = db.get_serann_by_generation(0)
    assert list(back.index) == ["a", "b"] and back.loc["b", "is_valid"] == False  # noqa: E712
    db.save_generation_info({"experiment_id": "e", "generation": 0})
    assert db.get_generations_count() == 1
    nxt = pd.DataFrame({"genotype": [np.zeros(4)], "parent_id": ["a"]}, index=pd.Index(["c"], name="id"))
    db.save_resume_state(0, {"next_generation": nxt, "pool_size": 3, "rng": None})
    st = db.get_resume_state(0)
    assert st["pool_size"] == 3 and list(st["next_generation"].index) == ["c"] and "rng" not in st
    assert db.get_resume_state(1) is None
