"""Assembly of an experiment from parameters: data, codec, engine, communicator, DB.

Used by the CLI (``evolutionary_experiment/run_experiment.py``), ``bench.py`` and the tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..config import experiment_config
from ..data.datasets import get_serann_data, load_encodings, load_mnist
from ..engine.base import TrainConfig
from ..genome.codec import TableCodec
from ..parallel.comm import Comm, make_comm
from .worker import ShardWorker


def default_device(comm: Comm):
    import torch
    if torch.cuda.is_available():
        idx = comm.local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(idx)
        return f"cuda:{idx}"
    return "cpu"


def default_engine(device: str) -> str:
    """CPU: the torch engine.  GPU: the HIP engine, and a loud error when its extension is missing --
    a silent eager fallback would report eager-PyTorch numbers as the framework's (the torch engine on
    a GPU stays available explicitly: ``--engine torch`` / ``SERANN_ENGINE=torch``)."""
    if not str(device).startswith("cuda"):
        return "torch"
    forced = os.environ.get("SERANN_ENGINE")
    if forced:
        return forced
    from ..ops import hip_ops
    if not hip_ops.available():
        raise RuntimeError("serann_hip extension not loadable on a GPU device: build it in-tree first "
                           "(python -c 'import __graft_entry__ as g; g.build()'), or pass --engine torch")
    return "hip"


def build_codec(parameters: dict, codec: str = "auto", table_size: int = 4096, seed: int = 0,
                device: str = "cpu", sensitive_bits: Optional[int] = None):
    """``auto``: the RiboAE checkpoint named in the config when it exists, else the synthetic table
    codec."""
    if codec in ("auto", "riboae"):
        path = experiment_config["ribosomal_autoencoder_path"]
        ckpt = path if path.endswith(".pt") else path + ".pt"
        if os.path.exists(ckpt):
            from ..riboae.io import load_codec
            return load_codec(ckpt, experiment_config["vocabulary_path"], device=device,
                              max_tokens=int(parameters["max_tokens"]))
        if codec == "riboae":
            raise FileNotFoundError(f"RiboAE checkpoint not found: {ckpt}")
    return TableCodec.from_generator(table_size, seed=seed, genotype_size=int(parameters["genotype_size"]),
                                     ancestor=parameters.get("ancestor_genotype"),
                                     sensitive_bits=sensitive_bits)


@dataclass
class Setup:
    comm: Comm
    device: str
    engine: str
    codec: object
    encodings: np.ndarray
    data: object
    worker: ShardWorker


def setup(parameters: dict, engine: str = "auto", codec: str = "auto", comm: Optional[Comm] = None,
          n_train: Optional[int] = None, n_test: Optional[int] = None, device: Optional[str] = None,
          train_cfg: Optional[TrainConfig] = None, table_size: int = 4096) -> Setup:
    comm = comm or make_comm()
    device = device or default_device(comm)
    from .capacity import admit
    admit(device)                       # GPU-memory admission (reference run_experiment.py:103)
    if engine == "auto":
        engine = default_engine(device)
    encodings = load_encodings(genotype_size=int(parameters["genotype_size"]))
    data = get_serann_data(encodings, load_mnist(), int(parameters["num_classification_classes"]),
                           n_train=n_train, n_test=n_test)
    cdc = build_codec(parameters, codec, table_size=table_size, device=device)
    cfg = train_cfg or TrainConfig(epochs=int(parameters["training_epochs"]),
                                   batch_size=int(parameters["training_batch_size"]))
    worker = ShardWorker(parameters, data, engine=engine, device=device, train_cfg=cfg)
    return Setup(comm, device, engine, cdc, encodings, data, worker)
