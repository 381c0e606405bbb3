#!/usr/bin/env python
"""Tutorial (script form of the reference's synthetic_serann_generator/tutorial.ipynb).

1. Generate a synthetic SeRANN dataset with the layer-transition Markov chain and look at its
   distributions: token length, parameter count, layers per branch, loss_balance, validity (notebook
   cells at tutorial.ipynb:44-3516).
2. Train one SeRANN on MNIST classification + genotype replication and report its validation accuracy
   and replication fidelity (notebook cells at tutorial.ipynb:3527-3702; the notebook trains one net
   with Adadelta at batch 32 -- here the experiment's own settings: Keras Adam, batch 750).

    python synthetic_serann_generator/tutorial.py [--n 2000] [--epochs 1] [--device cuda]

MNIST is read from data/mnist.npz when present, otherwise a synthetic MNIST-shaped set is used (no network).
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def _hist(name, values, bins=10):
    values = np.asarray(values, dtype=np.float64)
    if len(values) == 0:
        print(f"{name}: (empty)")
        return
    counts, edges = np.histogram(values, bins=bins)
    top = max(1, counts.max())
    print(f"\n{name}: n={len(values)} mean={values.mean():.4g} median={np.median(values):.4g}")
    for c, lo, hi in zip(counts, edges[:-1], edges[1:]):
        print(f"  [{lo:12.4g}, {hi:12.4g})  {c:6d}  {'#' * int(40 * c / top)}")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000, help="synthetic nets to generate")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--device", default=None)
    ap.add_argument("--max-steps", type=int, default=None, help="steps per epoch cap (quick runs only)")
    a = ap.parse_args(argv)

    import torch
    from serann.config import default_parameters
    from serann.data.datasets import get_serann_data, load_encodings
    from serann.engine.base import TrainConfig
    from serann.experiment.worker import make_engine
    from serann.analysis.results import print_code, replication_fidelity
    from serann.genome.codec import decoded_form
    from serann.genome.generator import generate
    from serann.genome.interpreter import layer_counts, try_interpret
    from serann.genome.tokenizer import tokenize

    params = default_parameters("example")
    L = int(params["genotype_size"])
    # ---- 1. the synthetic dataset -------------------------------------------------------------
    df = generate(a.n, seed=a.seed)
    print(f"generated {len(df)} unique nets; columns: {list(df.columns)}")
    _hist("token length", [len(tokenize(s)) for s in df["code"]])
    _hist("parameters (generator count, genotype length 350)", df["parameters_count"])
    _hist("loss_balance", df["loss_balance"])
    results = [try_interpret(decoded_form(s), genotype_size=L) for s in df["code"]]
    ok = [r for r in results if r.ok]
    trainable = [r for r in ok if r.parameters_count <= float(params["max_serann_parameters"])]
    print(f"\nvalid at genotype length {L}: {len(ok)}/{len(results)}; trainable (<= "
          f"{params['max_serann_parameters']:.0f} parameters): {len(trainable)}")
    counts = [layer_counts(decoded_form(s)) for s, r in zip(df["code"], results) if r.ok]
    for name in ("classification", "replication", "merged"):
        _hist(f"{name} layers", [c[f"{name}_layers"] for c in counts], bins=6)

    # ---- 2. train one SeRANN ------------------------------------------------------------------
    pick = min(trainable, key=lambda r: abs(r.parameters_count - 1e6))
    src = next(s for s, r in zip(df["code"], results) if r is pick)
    print("\nthe net trained below:\n")
    print_code(src)
    dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    engine = "hip" if dev.startswith("cuda") else "torch"
    data = get_serann_data(load_encodings(None, n=70000, genotype_size=L))
    cfg = TrainConfig(epochs=a.epochs, batch_size=int(params["training_batch_size"]),
                      max_steps_per_epoch=a.max_steps)
    eng = make_engine(engine, [pick.ir], [a.seed], dev, cfg)
    fit = eng.fit(data, cfg)
    test_acc = eng.evaluate(data.test_x, data.test_labels, data.test_g, cfg)
    n_rep = 32
    rep = eng.replicate(np.asarray(data.test_g[:1], np.float32), [data.test_x[:n_rep]], cfg)[0]
    fid = replication_fidelity(np.repeat(data.test_g[:1], n_rep, 0), rep)
    eng.close()
    print(f"\n{engine} engine on {dev}: {fit.steps} steps in {fit.learning_time:.2f} s; "
          f"validation accuracy {float(fit.val_acc[0]):.4f}, test accuracy {float(test_acc[0]):.4f}; "
          f"replication fidelity {fid:.1f} / {L} loci; loss_balance {pick.ir.loss_balance:.4f}")
    return dict(valid=len(ok), trainable=len(trainable), val_acc=float(fit.val_acc[0]), fidelity=fid)


if __name__ == "__main__":
    main()
