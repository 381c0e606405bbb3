"""Bitwise reproducibility of one training step: runs HipPopulationEngine.debug_train_step ``--trials`` times on
the same batch and weights and prints, per organism and parameter tensor, the gradient elements that ever differ
from the first trial (GPU diagnostic)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from serann.engine.base import TrainConfig  # noqa: E402
from serann.engine.hip_engine import HipPopulationEngine  # noqa: E402
from serann.genome.interpreter import interpret  # noqa: E402
from tests.archs import ARCHS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--archs", default="")
    a = ap.parse_args()
    names = sorted(ARCHS) if not a.archs else a.archs.split(",")
    irs = [interpret(ARCHS[n]) for n in names]
    eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=TrainConfig(batch_size=a.batch))
    rng = np.random.default_rng(0)
    x = rng.random((a.batch, 28, 28, 1), dtype=np.float32)
    g = rng.integers(0, 2, (a.batch, 100)).astype(np.float32)
    y = rng.integers(0, 10, a.batch)
    ref, _ = eng.debug_train_step(x, g, y)
    ref = ref.cpu()
    bad = torch.zeros_like(ref, dtype=torch.bool)
    for _ in range(a.trials - 1):
        gr, _ = eng.debug_train_step(x, g, y)
        bad |= gr.cpu() != ref
    print("trials", a.trials, "differing gradient elements:", int(bad.sum()), "of", bad.numel())
    for o, (n, L) in enumerate(zip(names, eng.layouts)):
        offs = sorted([(off, kind, nid) for kind in ("w", "b", "gamma", "beta") for nid, off in getattr(L, kind).items()])
        for i, (off, kind, nid) in enumerate(offs):
            end = offs[i + 1][0] if i + 1 < len(offs) else off + 1
            seg = bad[off:end]
            if seg.any():
                idx = torch.nonzero(seg).flatten()[:8].tolist()
                print(f"org {o} {n} {kind}[{nid}] {L.ir.node(nid).attrs.get('kind')}: {int(seg.sum())} differ, first {idx}")


if __name__ == "__main__":
    main()
