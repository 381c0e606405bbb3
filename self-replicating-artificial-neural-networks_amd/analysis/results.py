"""Analysis utilities (reference: common/utils.py:17-412).

* ``load_experiment_results``     -- SQL -> DataFrame with ``genotype_hex``, ``is_mutant``, ``descendants``
                                     and ``parent_*`` columns, cached as a pickle under ``data_cache_dir``;
                                     reads the current ``serann`` table and the legacy ``srann`` table the
                                     reference's loader expects.
* ``load_experiment_data``        -- the same frame loaded by DB *path*, without ``parent_*`` columns,
                                     optionally joined with deep-evaluation columns by ``genotype_hex``.
* ``load_experiment_evaluations`` -- fitness algebra w = V*f*N, W = V*F over deep evaluations.
* ``load_deep_evaluations``       -- evaluation CSV joined with experiment rows and parents.
* ``prepare_muller_plot_data``    -- clone identity tracking (IBS) and dominant-clone frames.
* ``print_code``                  -- syntax-highlighted source (pygments).
* ``get_serann_model``            -- a single organism as a trainable torch module (oracle engine).

The absolute-fertility column is ``absolute_fertility`` in the current schema and
``absolute_fitness`` in the legacy one; both are accepted.
"""
from __future__ import annotations

import ast
import os
import pickle
import sqlite3
from pathlib import Path
from typing import Optional

import numpy as np
import pandas as pd

from ..config import global_config as config


def print_code(source_code: str):
    try:
        from pygments import highlight
        from pygments.formatters import TerminalTrueColorFormatter
        from pygments.lexers import PythonLexer
        print(highlight(source_code, PythonLexer(), TerminalTrueColorFormatter(style="autumn")))
    except ImportError:  # pragma: no cover
        print(source_code)


def genotype_to_hex(genotype) -> str:
    bits = "".join(str(int(b)) for b in np.asarray(genotype).astype(int).ravel())
    return hex(int(bits, 2)) if bits else hex(0)


def _parse_genotype(s: str) -> np.ndarray:
    return np.array(ast.literal_eval(s.replace("nan", "None")), dtype=float).astype(int)


def _serann_table(conn) -> str:
    names = {r[0] for r in conn.execute("select name from sqlite_master where type='table'")}
    if "serann" in names:
        return "serann"
    if "srann" in names:
        return "srann"
    raise ValueError("no serann/srann table in the experiment DB")


def _fertility_column(df: pd.DataFrame) -> str:
    return "absolute_fertility" if "absolute_fertility" in df.columns else "absolute_fitness"


def load_experiment_results(results_name: str, evaluations_name: Optional[str] = None, cache_invalidate: bool = False,
                            db_path: Optional[str] = None, **evaluations_params) -> pd.DataFrame:
    cache_path = Path(config["data_cache_dir"]) / "experiment_results" / f"{results_name}.pkl"
    if not cache_invalidate and cache_path.is_file():
        with open(cache_path, "rb") as f:       # written by this function (our own file)
            results = pickle.load(f)
    else:
        db_path = db_path or str(Path(config["experiment_results_dir"]) / f"{results_name}.sqlite")
        conn = sqlite3.connect(db_path)
        table = _serann_table(conn)
        df = pd.read_sql(f"select * from {table}", conn).set_index("id")
        conn.close()
        logical = {s: _parse_genotype(s) for s in df["genotype"].unique()}
        df["genotype_hex"] = df["genotype"].map(lambda s: genotype_to_hex(logical[s]))
        df["genotype"] = df["genotype"].map(lambda s: logical[s])
        df["is_mutant"] = df["genotype_hamming_distance_from_parent"] > 0
        descendants = {}
        pairs = df.dropna(subset=["parent_id"]).iloc[::-1]["parent_id"]
        for _id, parent_id in zip(pairs.index, pairs.values):
            descendants[parent_id] = descendants.get(parent_id, 0) + descendants.get(_id, 0) + 1
        df["descendants"] = pd.Series(descendants, index=df.index).fillna(0)
        results = df
        cache_path.parent.mkdir(parents=True, exist_ok=True)
        with open(cache_path, "wb") as f:
            pickle.dump(results, f)
    if evaluations_name is not None:
        ev = load_experiment_evaluations(evaluations_name, results, cache_invalidate, **evaluations_params)
        results = results.join(ev.drop(columns=["id"]).drop_duplicates(subset=["genotype_hex"]).set_index("genotype_hex"),
                               on="genotype_hex", how="left")
    results = results.join(results.rename(columns={c: f"parent_{c}" for c in results.columns}), on="parent_id")
    results.loc[results["parent_id"].isna(), "parent_genotype_hex"] = "experiment_ancestor_genotype_hex"
    results.loc[results["parent_id"].isna(), "parent_id"] = "experiment_ancestor_id"
    return results


DEEP_EVALUATION_COLUMNS = ["classification_accuracy", "mutation_rate", "offspring_viability", "fecundity",
                           "normed_fecundity", "fitness"]


def load_experiment_data(path: str, deep_evaluations=None, force_download: bool = False,
                         cache_invalidate: bool = False) -> pd.DataFrame:
    """Per-organism frame of one experiment DB given by path (reference common/utils.py:199-258).

    Columns: every ``serann`` (or legacy ``srann``) column, ``genotype`` as an int array, ``genotype_hex``,
    ``is_mutant``, ``descendants`` (transitive descendant count); generation-0 rows get
    ``parent_id = 'experiment_ancestor_id'`` and ``parent_genotype_hex = 'experiment_ancestor_genotype_hex'``
    (the reference's boolean-mask assignment of those two raises in pandas; ``.loc`` is what it means).
    ``deep_evaluations``: a DataFrame or CSV path with ``genotype_hex`` and any of
    DEEP_EVALUATION_COLUMNS, left-joined on ``genotype_hex`` (first row per genotype).  The frame is
    cached under ``data_cache_dir`` by DB file name; ``cache_invalidate`` / ``force_download`` rebuild it.
    """
    cache_path = Path(config["data_cache_dir"]) / "experiment_data" / (Path(path).name + ".pkl")
    if not (cache_invalidate or force_download) and cache_path.is_file():
        with open(cache_path, "rb") as f:       # written by this function (our own file)
            results = pickle.load(f)
    else:
        name = Path(path).stem
        results = load_experiment_results(name, cache_invalidate=True, db_path=str(path))
        results = results[[c for c in results.columns if not c.startswith("parent_") or c == "parent_id"]].copy()
        results["parent_genotype_hex"] = np.where(results["parent_id"] == "experiment_ancestor_id",
                                                  "experiment_ancestor_genotype_hex", None)
        cache_path.parent.mkdir(parents=True, exist_ok=True)
        with open(cache_path, "wb") as f:
            pickle.dump(results, f)
    if deep_evaluations is not None:
        ev = pd.read_csv(deep_evaluations) if isinstance(deep_evaluations, (str, os.PathLike)) else deep_evaluations
        cols = [c for c in DEEP_EVALUATION_COLUMNS if c in ev.columns]
        results = results.join(ev[cols + ["genotype_hex"]].drop_duplicates(subset=["genotype_hex"])
                               .set_index("genotype_hex"), on="genotype_hex", how="left")
    return results


def evaluations_from_pickle(path: str) -> pd.DataFrame:
    """Flatten a SampleDeepEvaluator output pickle into the CSV layout used by the analysis
    (serann_id, visited, classification_accuracy, mutation_rate, offspring_viability)."""
    with open(path, "rb") as f:                 # written by serann.evaluation (our own file)
        raw = pickle.load(f)
    rows = []
    for sid, ev in raw.items():
        if not ev:
            rows.append({"serann_id": sid, "visited": False})
            continue
        acc = np.nanmean(ev["classification_accuracy"]) if np.size(ev["classification_accuracy"]) else np.nan
        mr = _hist_mean(ev["mutation_rate"])
        ov = _hist_mean(ev["offspring_survival"])
        rows.append({"serann_id": sid, "visited": True, "classification_accuracy": acc, "mutation_rate": mr,
                     "offspring_viability": ov})
    return pd.DataFrame(rows)


def _hist_mean(hists) -> float:
    if isinstance(hists, dict):
        hists = [hists]
    num, den = 0.0, 0.0
    for h in hists or []:
        for k, v in h.items():
            num += float(k) * v
            den += v
    return num / den if den else np.nan


def load_experiment_evaluations(evaluations_name: str, experiment_results: pd.DataFrame, cache_invalidate=False,
                                selection_intensity: float = 1, raw_data: bool = False) -> pd.DataFrame:
    cache_path = Path(config["data_cache_dir"]) / "deep_evaluations" / f"{evaluations_name}.pkl"
    if not cache_invalidate and cache_path.is_file():
        with open(cache_path, "rb") as f:
            return pickle.load(f)
    base = Path(config["deep_evaluations_dir"])
    if raw_data:
        evaluations = evaluations_from_pickle(str(base / f"{evaluations_name}.pkl"))
    else:
        evaluations = pd.read_csv(base / f"{evaluations_name}.csv")
    evaluations = evaluations.rename(columns={"serann_id": "id"})
    evaluations = evaluations[evaluations["visited"] == True].drop(columns="visited")  # noqa: E712
    fcol = _fertility_column(experiment_results)
    res = experiment_results.loc[evaluations["id"].values, [fcol, "generation", "genotype_hex"]]
    evaluations = evaluations.merge(res, left_on="id", right_index=True).rename(
        columns={"classification_accuracy": "m_classification_accuracy", "mutation_rate": "m_mutation_rate"})
    evaluations["m_absolute_fertility"] = evaluations["m_classification_accuracy"].fillna(0) ** selection_intensity
    evaluations["m_offspring_survival"] = evaluations["offspring_viability"].fillna(0)
    sums = experiment_results.groupby("generation")[fcol].apply(lambda x: np.sum(x.fillna(0) ** selection_intensity))
    evaluations = evaluations.join(sums.rename("absolute_fertility_sum"), on="generation")
    # f = F^lambda / sum F_j^lambda
    evaluations["m_relative_fertility"] = evaluations["m_absolute_fertility"] / evaluations["absolute_fertility_sum"]
    pop_size = experiment_results.groupby("generation")["genotype"].count().max()
    # w(t) = V * f * N
    evaluations["m_relative_fitness"] = evaluations["m_offspring_survival"] * evaluations["m_relative_fertility"] * pop_size
    # W(t) = V * F
    evaluations["m_absolute_fitness"] = evaluations["m_offspring_survival"] * evaluations["m_absolute_fertility"]
    sl = experiment_results.loc[evaluations["id"].values]
    mask = ((sl["is_valid"] == False) | (sl["is_overweight"] == True)).values  # noqa: E712
    evaluations.loc[mask, "m_relative_fitness"] = 0
    evaluations.loc[mask, "m_absolute_fitness"] = 0
    cols = ["id", "genotype_hex", "m_classification_accuracy", "m_mutation_rate", "m_offspring_survival",
            "m_relative_fertility", "m_absolute_fertility", "m_absolute_fitness", "m_relative_fitness"]
    evaluations = evaluations[cols]
    cache_path.parent.mkdir(parents=True, exist_ok=True)
    with open(cache_path, "wb") as f:
        pickle.dump(evaluations, f)
    return evaluations


def load_deep_evaluations(sample_name: str, experiment_id: str, selection_intensity: float = 1) -> pd.DataFrame:
    evaluations = pd.read_csv(Path(config["deep_evaluations_dir"]) / f"{sample_name}.csv")
    evaluations = evaluations[evaluations["visited"] == True].drop(columns="visited")  # noqa: E712
    conn = sqlite3.connect(str(Path(config["experiment_results_dir"]) / f"{experiment_id}.sqlite"))
    table = _serann_table(conn)
    exp = pd.read_sql(f"select * from {table}", conn)
    conn.close()
    exp["genotype"] = exp["genotype"].map(_parse_genotype)
    exp["genotype_hex"] = exp["genotype"].map(genotype_to_hex)
    fcol = _fertility_column(exp)
    ev = evaluations.merge(exp, left_on="serann_id", right_on="id")
    parents = exp[exp["id"].isin(ev["parent_id"].dropna())].drop(columns="parent_id")
    parents.columns = ["parent_" + c for c in parents.columns]
    ev = ev.merge(parents, on="parent_id", how="left")
    ev["absolute_fecundity"] = ev["classification_accuracy"].fillna(0)
    ev["offspring_viability"] = ev["offspring_viability"].fillna(0)
    sums = exp.groupby("generation")[fcol].apply(lambda x: np.sum(x.fillna(0) ** selection_intensity))
    ev = ev.join(sums.rename("absolute_fecundity_sum"), on="generation")
    ev["fecundity"] = ev["absolute_fecundity"] ** selection_intensity / ev["absolute_fecundity_sum"]
    population_size = int((exp["generation"] == 0).sum())
    ev["normed_fecundity"] = population_size * ev["fecundity"]
    ev["fitness"] = ev["offspring_viability"] * ev["fecundity"] * population_size
    ev.loc[(ev["is_valid"] == False) | (ev["is_overweight"] == True), "fitness"] = 0  # noqa: E712
    return ev


def prepare_muller_plot_data(df: pd.DataFrame, ancestor_id: Optional[str] = None, frequency_threshold: float = 0.3,
                             return_identity_map: bool = False):
    """Clone identities (identical by state: same parent identity + same genotype), dominant clones
    above ``frequency_threshold`` x population, population and adjacency frames for Muller plots."""
    df = df.copy()
    ancestor_id = ancestor_id or df[df["generation"] == 0].iloc[0].name
    df = df.reset_index()
    df.loc[df["generation"] == 1, "parent_id"] = ancestor_id
    df.loc[df["generation"] == 0, "id"] = ancestor_id
    df = df.drop_duplicates(subset="id").set_index("id")
    population_size = len(df[df["generation"] == 1])
    counts = df.groupby("parent_id")["genotype"].count().reindex(df.index, fill_value=0)
    df["offspring_counts"] = counts
    keep = df.groupby("genotype_hex")["offspring_counts"].transform("max") > 0
    df = df[keep | (df.index == ancestor_id)].copy()
    df["identity"] = 1
    df["parent_identity"] = np.nan
    next_identity = 2
    for generation in sorted(df["generation"].unique()):
        if generation == 0:
            continue
        data = df[df["generation"] == generation]
        parent_ident = df.loc[data["parent_id"], "identity"].values
        same = (data["genotype_hex"].values == df.loc[data["parent_id"], "genotype_hex"].values)
        df.loc[data.index, "parent_identity"] = parent_ident
        df.loc[data.index[same], "identity"] = parent_ident[same]
        diff_idx = data.index[~same]
        groups = {}
        for i, pid, gh in zip(diff_idx, parent_ident[~same], data.loc[diff_idx, "genotype_hex"]):
            key = (pid, gh)
            if key not in groups:
                groups[key] = next_identity
                next_identity += 1
            df.at[i, "identity"] = groups[key]
    max_freq = df.groupby(["identity", "generation"])["genotype"].count().groupby(level=0).max()
    for parent_identity, off in df.sort_values("parent_identity", ascending=False).groupby("parent_identity", sort=False):
        cands = [parent_identity] + list(off["identity"].unique())
        max_freq.loc[parent_identity] = max(max_freq.reindex(cands).fillna(0))
    dominant = max_freq[max_freq > frequency_threshold * population_size]
    rows = df[df["identity"].isin(dominant.index)]
    pops = rows.groupby(["generation", "identity"])["genotype"].count()
    idx = pd.MultiIndex.from_product([sorted(rows["generation"].unique()), dominant.index],
                                     names=["generation", "identity"])
    pops = pops.reindex(idx, fill_value=0)
    for g in sorted(rows["generation"].unique()):
        pops.loc[(g, 0)] = population_size - pops.loc[g].sum()
    pops = pops.sort_index().reset_index()
    pops.columns = ["Generation", "Identity", "Population"]
    adj = rows.groupby("identity")["parent_identity"].min().reset_index().rename(
        columns={"identity": "Identity", "parent_identity": "Parent"})
    adj = adj.fillna({"Parent": 0})
    adj = adj[adj["Identity"] != adj["Parent"]][["Parent", "Identity"]]
    if return_identity_map:
        return pops, adj, df["identity"]
    return pops, adj


def get_serann_model(source_code: str, seed: int = 0, device: str = "cpu", genotype_size: int = 100):
    """Single organism on the oracle engine (reference: common/utils.py:21-54 ``get_serann_keras_model``).
    Returns (module, ir); ``module(x, g, training)`` -> (class logits, replication logits)."""
    from ..genome.interpreter import interpret
    from ..models.organism import Organism, init_params
    ir = interpret(source_code, genotype_size=genotype_size)
    return Organism(ir, init_params(ir, seed), device=device), ir


def replication_fidelity(target: np.ndarray, pred: np.ndarray) -> float:
    """Mean number of correctly copied loci (the notebook metric)."""
    p = np.clip(np.round(pred), 0, 1)
    return float(np.mean(np.sum(p == target, axis=1)))
