"""Configuration tiers (reference: global_config.py:6-18,
evolutionary_experiment/config.py:4-17, ribosomal_autoencoder/config.py:4-10).

Three tiers are kept: (1) python dicts with the same keys as the reference,
(2) JSON parameter files (loaded unchanged), (3) CLI flags.  Paths can be
overridden with ``SERANN_ROOT`` (project root) or per-key environment variables
``SERANN_<KEY_UPPER>``.

``max_serann_per_gpu`` (112, a V100-era job size) is kept as a key for compatibility
but not applied: a rank trains its whole shard at once when it fits in HBM and in
waves sized from each organism's estimated device bytes otherwise
(:mod:`serann.experiment.capacity`).  ``worker_pool_job_timeout`` is the
per-generation watchdog timeout (:class:`serann.utils.faults.GenerationWatchdog`)
and sets the collective timeout.
"""
from __future__ import annotations

import json
import os
import tempfile
from pathlib import Path

_package_root = Path(__file__).resolve().parent
_project_root = Path(os.environ.get("SERANN_ROOT", _package_root.parent))


def _p(*parts) -> str:
    return str(Path(_project_root, *parts))


global_config = {
    "workers_pool_port": 6379,
    "project_root": _project_root,
    "experiment_results_dir": _p("data", "experiment_results"),
    "synthetic_datasets_dir": _p("data", "synthetic_datasets"),
    "token_sequences_dir": _p("data", "token_sequences"),
    "vocabularies_dir": _p("data", "vocabularies"),
    "encodings_datasets_dir": _p("data", "encodings_datasets"),
    "evaluation_db": _p("data", "evaluation_db.sqlite"),
    "ribosomal_autoencoders_dir": _p("models", "ribosomal_autoencoder"),
    "serann_evaluations_dir": _p("data", "serann_evaluations"),
    # referenced but never defined by the reference
    "deep_evaluations_dir": _p("data", "serann_evaluations"),
    "mnist_path": _p("data", "mnist.npz"),
    "data_cache_dir": str(Path(tempfile.gettempdir()) / "serann_cache"),
}

experiment_config = dict(global_config)
experiment_config.update({
    "worker_pool_job_timeout": 1080,
    "max_serann_per_gpu": 112,
    "encodings_dataset_path": str(Path(global_config["encodings_datasets_dir"],
                                       "generated_27032020__sloppy-cornflower-dane_b69079.npz")),
    "vocabulary_path": str(Path(global_config["vocabularies_dir"], "generated_27032020.csv")),
    "ribosomal_autoencoder_path": str(Path(global_config["ribosomal_autoencoders_dir"],
                                           "sloppy-cornflower-dane_b69079")),
    "random_seed": 79375,
})

riboae_config = dict(global_config)
riboae_config.update({
    "half_precision": True,
    "token_sequences_dataset_path": str(Path(global_config["token_sequences_dir"], "generated_27032020.npz")),
    "vocabulary_path": str(Path(global_config["vocabularies_dir"], "generated_27032020.csv")),
    "random_seed": 534213,
})


def _apply_env_overrides(cfg: dict) -> dict:
    for key in list(cfg):
        env = os.environ.get("SERANN_" + key.upper())
        if env is not None:
            cfg[key] = type(cfg[key])(env) if isinstance(cfg[key], (int, float)) else env
    return cfg


for _cfg in (global_config, experiment_config, riboae_config):
    _apply_env_overrides(_cfg)

# default parameter files shipped with the package (same schema as the reference)
PARAMETERS_DIR = _package_root / "parameters"


def load_parameters(path) -> dict:
    """Load a JSON parameter file (C04-C06 schema)."""
    with open(path, "r") as f:
        return json.load(f)


def default_parameters(name: str = "example") -> dict:
    return load_parameters(PARAMETERS_DIR / "experiment" / f"{name}.json")
