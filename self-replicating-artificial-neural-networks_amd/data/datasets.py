"""Datasets: MNIST (or an MNIST-shaped synthetic stand-in) and genotype encodings.

Reference semantics (common/logic.py:38-55, experiment_worker.py:197-220):

* images ``x/255`` shaped (N, 28, 28, 1); one-hot labels shaped (N, 1, 10);
* genotypes ``encodings[:60000]`` are both the replication input (N, 100, 1) and its target
  (N, 1, 100); the test split uses ``encodings[60000:70000]``.

There is no network access, so ``keras.datasets.mnist`` is replaced by ``load_mnist``: it reads a
local ``mnist.npz`` (keys ``x_train y_train x_test y_test``) when one exists and otherwise builds a
deterministic, *learnable* synthetic MNIST-shaped dataset (class prototypes + noise).  Results
obtained on the synthetic data say so (``data: "synthetic"``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..config import experiment_config, global_config


@dataclass
class MnistData:
    x_train: np.ndarray   # uint8 (60000, 28, 28)
    y_train: np.ndarray   # int64 (60000,)
    x_test: np.ndarray    # uint8 (10000, 28, 28)
    y_test: np.ndarray    # int64 (10000,)
    synthetic: bool


def synthetic_mnist(n_train=60000, n_test=10000, shape=(28, 28), classes=10, seed=1234, label_noise=0.03,
                    mix=0.15) -> MnistData:
    """MNIST-shaped synthetic classification data (no network access for the real set).

    Every image is its class prototype (a smooth random field), blended with a random other class's prototype
    (weight ~ U(0, ``mix``): some overlap between classes, like confusable digits), scaled, plus pixel noise; a fraction
    ``label_noise`` of the labels is replaced by a random class.  Without the blending and label noise
    (round 4) every organism reached 0.98-1.0 validation accuracy, so fertility = accuracy^lambda was almost
    flat and the benched populations drifted rather than evolved; with them good models plateau near MNIST's
    ~0.97 (the reference tutorial's single SeRANN, tutorial.ipynb:3702: 3 % label noise caps accuracy at ~0.973)
    and selection has something to act on.  (mix = 0.45 left the bench population at 0.88-0.90.)"""
    rng = np.random.default_rng(seed)
    h, w = shape
    # smooth class prototypes: low-frequency random fields
    yy, xx = np.meshgrid(np.linspace(-1, 1, h), np.linspace(-1, 1, w), indexing="ij")
    protos = []
    for _ in range(classes):
        f = np.zeros((h, w))
        for _ in range(4):
            a, b, c, d = rng.normal(size=4)
            f += np.sin(2.5 * a * xx + 2.5 * b * yy + c) * d
        f = (f - f.min()) / (np.ptp(f) + 1e-9)
        protos.append(f)
    protos = np.stack(protos)

    def make(n, rng):
        y = rng.integers(0, classes, size=n)
        scale = rng.uniform(0.6, 1.0, size=(n, 1, 1))
        noise = rng.normal(0, 0.25, size=(n, h, w))
        other = (y + rng.integers(1, classes, size=n)) % classes
        a = rng.uniform(0.0, mix, size=(n, 1, 1))
        x = np.clip(((1 - a) * protos[y] + a * protos[other]) * scale + noise, 0, 1)
        flip = rng.random(n) < label_noise
        y = np.where(flip, rng.integers(0, classes, size=n), y)
        return (x * 255).astype(np.uint8), y.astype(np.int64)

    xt, yt = make(n_train, rng)
    xs, ys = make(n_test, rng)
    return MnistData(xt, yt, xs, ys, synthetic=True)


def load_mnist(path: Optional[str] = None, allow_synthetic: bool = True, **synthetic_kw) -> MnistData:
    path = path or global_config["mnist_path"]
    if path and os.path.isfile(path):
        with np.load(path, allow_pickle=False) as f:
            return MnistData(f["x_train"], f["y_train"].astype(np.int64), f["x_test"],
                             f["y_test"].astype(np.int64), synthetic=False)
    if not allow_synthetic:
        raise FileNotFoundError(f"MNIST not found at {path}")
    return synthetic_mnist(**synthetic_kw)


def synthetic_encodings(n=70000, genotype_size=100, seed=4321) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.integers(0, 2, size=(n, genotype_size)).astype(np.int8)


def load_encodings(path: Optional[str] = None, allow_synthetic: bool = True, n: int = 70000,
                   genotype_size: int = 100) -> np.ndarray:
    path = path or experiment_config["encodings_dataset_path"]
    if path and os.path.isfile(path):
        with np.load(path, allow_pickle=False) as f:
            return f["encodings"]
    if not allow_synthetic:
        raise FileNotFoundError(f"encodings dataset not found at {path}")
    return synthetic_encodings(n, genotype_size)


@dataclass
class SerannData:
    """Host-side training/test arrays in reference layout (float32)."""
    train_x: np.ndarray        # (N, H, W, 1)  x/255
    train_labels: np.ndarray   # (N,) int
    train_g: np.ndarray        # (N, L)  {0,1}
    test_x: np.ndarray
    test_labels: np.ndarray
    test_g: np.ndarray
    num_classes: int
    synthetic: bool

    @property
    def n_train(self) -> int:
        return len(self.train_x)


def get_serann_data(encodings: np.ndarray, mnist: Optional[MnistData] = None, num_classes: int = 10,
                    n_train: Optional[int] = None, n_test: Optional[int] = None) -> SerannData:
    """Build the joint training data (common/logic.py:38-55).  ``n_train``/``n_test`` subsample
    for CPU tests only."""
    mnist = mnist or load_mnist()
    xtr = mnist.x_train.astype(np.float32)[..., None] / 255.0
    xte = mnist.x_test.astype(np.float32)[..., None] / 255.0
    ntr, nte = len(xtr), len(xte)
    g_train = encodings[:ntr].astype(np.float32)
    g_test = encodings[ntr:ntr + nte].astype(np.float32)
    if len(g_train) < ntr or len(g_test) < nte:
        raise ValueError(f"encodings dataset needs >= {ntr + nte} rows (has {len(encodings)})")
    d = SerannData(xtr, mnist.y_train, g_train, xte, mnist.y_test, g_test, num_classes, mnist.synthetic)
    if n_train is not None:
        d.train_x, d.train_labels, d.train_g = d.train_x[:n_train], d.train_labels[:n_train], d.train_g[:n_train]
    if n_test is not None:
        d.test_x, d.test_labels, d.test_g = d.test_x[:n_test], d.test_labels[:n_test], d.test_g[:n_test]
    return d
