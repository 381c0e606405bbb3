"""SQLite experiment database (reference: evolutionary_experiment/logic/experiment_db.py:7-125).

Same tables and column names as the reference writer: ``execution_info`` (rewritten
with ``if_exists='replace'`` after appending one row per run/resume), ``serann`` (appended per
generation, index ``id``), ``generations`` (one row per generation), ``model_metrics``.

Differences (documented): uses the stdlib ``sqlite3`` driver (pandas' sqlite fallback) instead of
SQLAlchemy; DB errors are *raised* unless ``swallow_errors=True`` (the reference prints and
continues); an additive ``resume_state`` table stores the packed offspring
genotypes and RNG state so that resume is exact without retraining.  The resume state is
plain data -- a JSON text column and an ``.npz`` blob read with ``allow_pickle=False`` -- so opening a
shared results DB never unpickles anything.
"""
from __future__ import annotations

import ast
import io
import json
import sqlite3
from contextlib import contextmanager

import numpy as np
import pandas as pd

INT_COLUMNS = ["genotype_size", "initial_offspring_pool_size", "max_serann_parameters",
               "max_serann_tokens", "num_classification_classes", "num_generations", "num_seranns",
               "offspring_pool_size_factor", "random_seed", "training_batch_size", "training_epochs"]
FLOAT_COLUMNS = ["error_correction_probability", "selection_pressure"]


def _ts(v):
    """Timestamps are stored as pandas writes datetime64 columns: 'YYYY-MM-DD HH:MM:SS.ffffff'."""
    try:
        return pd.Timestamp(v).strftime("%Y-%m-%d %H:%M:%S.%f")
    except (TypeError, ValueError):
        return v


class ExperimentDB:
    def __init__(self, db_path, swallow_errors: bool = False):
        self._db_path = str(db_path)
        self._swallow = swallow_errors

    @property
    def db_path(self):
        return self._db_path

    @contextmanager
    def db_connection(self):
        conn = sqlite3.connect(self._db_path, timeout=60)
        try:
            yield conn
            conn.commit()
        except Exception:
            if not self._swallow:
                raise
            print("\033[91mFailed to access DB file\033[0m")
        finally:
            conn.close()

    @staticmethod
    def _table_exists(conn, name) -> bool:
        cur = conn.execute("select name from sqlite_master where type='table' and name=?", (name,))
        return cur.fetchone() is not None

    # ---- writers -------------------------------------------------------------------------------
    def save_execution_info(self, start_time, parameters: dict):
        row = {"start_time": _ts(start_time)}
        row.update(parameters)
        if "ancestor_genotype" in parameters and parameters["ancestor_genotype"] is not None:
            row["ancestor_genotype"] = "".join(str(int(i)) for i in row["ancestor_genotype"])
        if "classification_image_dimensions" in parameters:
            row["classification_image_dimensions"] = str(list(parameters["classification_image_dimensions"]))
        row = {k: (json.dumps(v) if isinstance(v, (list, dict)) else v) for k, v in row.items()}
        with self.db_connection() as conn:
            existing = pd.read_sql("select * from execution_info", conn) \
                if self._table_exists(conn, "execution_info") else pd.DataFrame()
            rows = pd.concat([existing, pd.DataFrame([row])], ignore_index=True)
            rows.to_sql("execution_info", conn, index=False, if_exists="replace")

    def save_seranns_info(self, seranns_info: pd.DataFrame):
        df = seranns_info.copy()
        df["genotype"] = df["genotype"].map(lambda x: str(np.asarray(x).tolist()))
        for c in ("is_valid", "is_overweight"):
            if c in df:
                df[c] = df[c].astype(object).where(df[c].notna(), None)
        with self.db_connection() as conn:
            df.to_sql("serann", conn, if_exists="append", index=True, index_label="id")

    def save_generation_info(self, generation_info: dict):
        generation_info = {k: (_ts(v) if k == "start_time" else v) for k, v in generation_info.items()}
        with self.db_connection() as conn:
            pd.DataFrame([generation_info]).to_sql("generations", conn, index=False, if_exists="append")

    def save_model_metrics(self, model_name, metrics: pd.DataFrame):
        with self.db_connection() as conn:
            metrics.assign(model=model_name).to_sql("model_metrics", conn, index=False, if_exists="append")

    def save_resume_state(self, generation: int, state: dict):
        """Additive table: exact resume point after ``generation``.

        ``state``: ``next_generation`` (DataFrame indexed by id with a ``genotype`` column of arrays),
        ``pool_size``, ``rng`` (``RandomState.get_state()`` tuple), ``random_seed``."""
        meta, arrays = _pack_resume_state(state)
        buf = io.BytesIO()
        np.savez(buf, **arrays)
        with self.db_connection() as conn:
            if self._table_exists(conn, "resume_state") and "meta" not in self._columns(conn, "resume_state"):
                conn.execute("drop table resume_state")      # pre-plain-data format: never read
            conn.execute("create table if not exists resume_state "
                         "(generation integer primary key, meta text, arrays blob)")
            conn.execute("insert or replace into resume_state values (?, ?, ?)",
                         (int(generation), json.dumps(meta), buf.getvalue()))

    @staticmethod
    def _columns(conn, table):
        return [r[1] for r in conn.execute(f"pragma table_info({table})").fetchall()]

    # ---- readers -------------------------------------------------------------------------------
    def get_last_execution_info(self) -> pd.Series:
        with self.db_connection() as conn:
            if not self._table_exists(conn, "execution_info"):
                return pd.Series(dtype=object)
            raw = pd.read_sql("select * from execution_info order by start_time desc limit 1", conn).iloc[0].copy()
        for column in raw.keys():
            if column in INT_COLUMNS and pd.notna(raw[column]):
                raw[column] = int(float(raw[column]))
            elif column in FLOAT_COLUMNS and pd.notna(raw[column]):
                raw[column] = float(raw[column])
        if "classification_image_dimensions" not in raw and "classification_image_height" in raw:
            raw["classification_image_dimensions"] = [int(raw["classification_image_height"]),
                                                      int(raw["classification_image_width"])]
        elif "classification_image_dimensions" in raw:
            raw["classification_image_dimensions"] = [int(v) for v in
                                                      ast.literal_eval(str(raw["classification_image_dimensions"]))]
        if "ancestor_genotype" in raw and isinstance(raw["ancestor_genotype"], str):
            raw["ancestor_genotype"] = [int(s) for s in raw["ancestor_genotype"]]
        if "initial_offspring_pool_size" not in raw:
            raw["initial_offspring_pool_size"] = 10
        if "offspring_pool_size_factor" not in raw or raw["offspring_pool_size_factor"] == 1:
            raw["offspring_pool_size_factor"] = 3
        return raw

    def get_generations_count(self) -> int:
        with self.db_connection() as conn:
            if not self._table_exists(conn, "generations"):
                return 0
            return int(conn.execute("select count(*) from generations").fetchone()[0])

    def get_executions_count(self) -> int:
        with self.db_connection() as conn:
            if not self._table_exists(conn, "execution_info"):
                return 0
            return int(conn.execute("select count(*) from execution_info").fetchone()[0])

    def get_serann_by_generation(self, generation: int) -> pd.DataFrame:
        with self.db_connection() as conn:
            df = pd.read_sql("select * from serann where generation = ?", conn, params=(int(generation),))
        df = df.set_index("id")
        df["genotype"] = df["genotype"].map(
            lambda x: np.array(ast.literal_eval(x.replace("nan", "None")), dtype=np.float64))
        df["is_valid"] = df["is_valid"].astype(bool)
        return df

    def get_resume_state(self, generation: int):
        with self.db_connection() as conn:
            if not self._table_exists(conn, "resume_state") or "meta" not in self._columns(conn, "resume_state"):
                return None
            row = conn.execute("select meta, arrays from resume_state where generation = ?",
                               (int(generation),)).fetchone()
        if not row:
            return None
        with np.load(io.BytesIO(row[1]), allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files}
        return _unpack_resume_state(json.loads(row[0]), arrays)


def _json_value(v):
    if v is None or (isinstance(v, float) and np.isnan(v)):
        return None
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return None if np.isnan(v) else float(v)
    if isinstance(v, (np.bool_,)):
        return bool(v)
    return v


def _pack_resume_state(state: dict):
    df = state["next_generation"]
    other = [c for c in df.columns if c != "genotype"]
    meta = {"ids": [str(i) for i in df.index], "index_name": df.index.name,
            "columns": {c: [_json_value(v) for v in df[c].tolist()] for c in other},
            "column_order": list(df.columns), "pool_size": int(state["pool_size"]),
            "random_seed": None if state.get("random_seed") is None else int(state["random_seed"])}
    arrays = {"genotype": np.stack([np.asarray(g, np.float64) for g in df["genotype"]])
              if len(df) else np.zeros((0, 0))}
    rng = state.get("rng")
    if rng is not None:
        name, keys, pos, has_gauss, cached = rng
        meta["rng"] = {"name": str(name), "pos": int(pos), "has_gauss": int(has_gauss), "cached": float(cached)}
        arrays["rng_keys"] = np.asarray(keys, np.uint32)
    return meta, arrays


def _unpack_resume_state(meta: dict, arrays: dict) -> dict:
    import pandas as pd_
    ids = meta["ids"]
    df = pd_.DataFrame(index=pd_.Index(ids, name=meta.get("index_name")))
    for c in meta["column_order"]:
        if c == "genotype":
            df["genotype"] = [arrays["genotype"][i] for i in range(len(ids))]
        else:
            vals = meta["columns"][c]
            df[c] = [np.nan if v is None and c != "parent_id" else v for v in vals]
    out = {"next_generation": df, "pool_size": meta["pool_size"], "random_seed": meta.get("random_seed")}
    if "rng" in meta:
        r = meta["rng"]
        out["rng"] = (r["name"], arrays["rng_keys"], r["pos"], r["has_gauss"], r["cached"])
    return out
