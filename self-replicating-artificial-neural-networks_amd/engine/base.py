"""Population-engine contract shared by the torch oracle and the HIP grouped engine.

One engine instance trains one *shard* of a generation: P independent organisms that share the
input mini-batches (one permutation per epoch, as Keras' joint ``fit`` does: experiment_worker.py:
66-83, 114-119).  It implements the reference worker's device work:

* ``fit``        -- ``training_epochs`` epochs, batch ``training_batch_size``, ``validation_split``
                    (the last 5 % of the training arrays, not shuffled), per-organism loss
                    ``lb * CE + (1 - lb) * MSE``, Keras Adam(1e-3, eps=1e-4);
* ``evaluate``   -- test accuracy with BN moving statistics (experiment_worker.py:87);
* ``replicate``  -- sigmoid replication outputs of each organism on its *own* rows only
                    (O(P * pool) instead of the reference's O(P^2 * pool)).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np


@dataclass
class TrainConfig:
    epochs: int = 5
    batch_size: int = 750
    validation_split: float = 0.05
    lr: float = 1e-3
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-4                 # Keras epsilon set to 1e-4 (experiment_worker.py:37, 80)
    eval_batch: int = 2000
    seed: int = 0                     # permutation seed (shared by every organism of a generation)
    max_steps_per_epoch: Optional[int] = None   # CI/debug override only; never used by bench.py
    val_every_epoch: bool = True      # the reference validates after every epoch
    # Adam moment storage of the HIP engine: "16bit" (bf16 m + log16 v: 16-bit moments as the reference's fp16
    # floatx keeps them, experiment_worker.py:36-37,80; csrc/hip/common.h MOM_16) or "fp32" (the torch oracle is
    # always fp32); env SERANN_ADAM_MOMENTS overrides the default
    adam_moments: str = field(default_factory=lambda: os.environ.get("SERANN_ADAM_MOMENTS", "16bit"))

    def split(self, n: int) -> int:
        # keras train_validation_split: split_at = int(floor(n * (1 - validation_split)))
        return int(math.floor(n * (1.0 - self.validation_split)))

    def steps_per_epoch(self, n_train: int) -> int:
        s = math.ceil(n_train / self.batch_size)
        if self.max_steps_per_epoch is not None:
            s = min(s, self.max_steps_per_epoch)
        return s


@dataclass
class FitResult:
    train_acc: np.ndarray            # last-epoch running accuracy (Keras history semantics)
    val_acc: np.ndarray              # after the last epoch
    val_mse: np.ndarray              # after the last epoch (unweighted replication loss)
    learning_time: float = 0.0
    steps: int = 0
    extra: dict = field(default_factory=dict)


def epoch_permutation(seed: int, epoch: int, n: int) -> np.ndarray:
    rng = np.random.default_rng([seed, epoch, 0x5EA])
    return rng.permutation(n)


def replication_image_rows(position: int, pool: int, total_rows: int, n_images: int) -> np.ndarray:
    """Image index of each replication row of the organism at ``position`` (among the trainable
    organisms of a job).  Reference: ``np.repeat(x_test, ceil(total/len(x_test)))[:total]`` and
    rows ``[position*pool, (position+1)*pool)`` (experiment_worker.py:140-160)."""
    repeat = max(1, int(math.ceil(total_rows / n_images)))
    rows = np.arange(position * pool, (position + 1) * pool)
    return rows // repeat


class PopulationEngine:
    """Abstract engine."""

    num_organisms: int

    def fit(self, data, cfg: TrainConfig) -> FitResult:
        raise NotImplementedError

    def evaluate(self, x: np.ndarray, labels: np.ndarray, g: np.ndarray, cfg: TrainConfig) -> np.ndarray:
        raise NotImplementedError

    def replicate(self, genotypes: np.ndarray, images: List[np.ndarray], cfg: TrainConfig) -> List[np.ndarray]:
        """genotypes: (P, L); images[i]: (pool, H, W, 1) for organism i -> list of (pool, L)."""
        raise NotImplementedError

    def close(self):
        pass
