"""Fit quality of the binary-genotype factorisation against the GEMM path: ``--pop`` ancestor clones (different
seeds) trained for ``--epochs`` at batch 750 on the synthetic data, once with SERANN_BINARY_NBN=1 and once with 0;
prints mean / spread of validation accuracy and replication MSE, and the moving BN statistics of the genotype
pair (GPU diagnostic)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=32)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--population-file", default="populations/ancestor_pop125.json")
    a = ap.parse_args()
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine import hip_engine as he
    from serann.engine.base import TrainConfig
    from serann.genome.interpreter import try_interpret
    irs = [try_interpret(s).ir for s in json.load(open(a.population_file))][:a.pop]
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=60000, n_test=2000, seed=5),
                           n_train=60000, n_test=2000)
    cfg = TrainConfig(epochs=a.epochs, batch_size=750)
    res = {}
    for binary in (True, False):
        he.BINARY_NBN = binary
        eng = he.HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        r = eng.fit(data, cfg)
        st = eng.stats.cpu().numpy() if hasattr(eng, "stats") else None
        res[binary] = (r.val_acc, r.val_mse, st)
        print(f"binary={binary}: val_acc mean {np.nanmean(r.val_acc):.4f} sd {np.nanstd(r.val_acc):.4f}  "
              f"val_mse mean {np.nanmean(r.val_mse):.5f} sd {np.nanstd(r.val_mse):.5f}  "
              f"learning {r.learning_time:.2f} s", flush=True)
        eng.close()
    (a1, m1, s1), (a0, m0, s0) = res[True], res[False]
    print(f"paired diff (binary - gemm): val_acc {np.nanmean(a1 - a0):+.4f} +- {np.nanstd(a1 - a0):.4f}, "
          f"val_mse {np.nanmean(m1 - m0):+.5f} +- {np.nanstd(m1 - m0):.5f}")
    if s1 is not None and s0 is not None:
        d = np.abs(s1 - s0)
        print(f"moving statistics arena: max |diff| {d.max():.3g}, mean {d.mean():.3g}")


if __name__ == "__main__":
    main()
