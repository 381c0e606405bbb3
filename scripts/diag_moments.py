#!/usr/bin/env python
"""16-bit vs fp32 Adam moments on the test architecture corpus: per-organism validation accuracy after a 2-epoch
fit, against the chaos of the same fit under a 1e-3 relative learning-rate perturbation (fp32 moments)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
from serann.engine.base import TrainConfig
from serann.engine.hip_engine import HipPopulationEngine
from serann.genome.interpreter import interpret
from tests.archs import ARCHS


def main():
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=8000, n_test=500, seed=12),
                           n_train=8000, n_test=500)
    names = sorted(ARCHS)
    irs = [interpret(ARCHS[n]) for n in names]
    out = {}
    for tag, mode, lr in (("fp32", "fp32", 1e-3), ("16bit", "16bit", 1e-3), ("fp32_lr+1e-3", "fp32", 1.001e-3),
                          ("16bit_lr+1e-3", "16bit", 1.001e-3)):
        for epochs in (2, 4):
            cfg = TrainConfig(epochs=epochs, batch_size=256, adam_moments=mode, lr=lr)
            eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
            res = eng.fit(data, cfg)
            out[(tag, epochs)] = res.val_acc
            del eng
    for epochs in (2, 4):
        print(f"epochs={epochs}")
        for i, n in enumerate(names):
            print(f"{n:28s} " + " ".join(f"{t}={out[(t, epochs)][i]:.4f}" for t in
                                         ("fp32", "16bit", "fp32_lr+1e-3", "16bit_lr+1e-3")))
        for t in ("16bit", "fp32_lr+1e-3", "16bit_lr+1e-3"):
            d = out[(t, epochs)] - out[("fp32", epochs)]
            print(f"  {t}: mean diff {d.mean():+.4f}  max |diff| {np.abs(d).max():.4f}")


if __name__ == "__main__":
    main()
