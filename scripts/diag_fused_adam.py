"""Where do the fused-Adam and arena-pass fits differ?  Runs test_fused_adam_matches_the_arena_pass's two fits
(SERANN_FUSE_ADAM 1 / 0) for ``--steps`` optimizer steps and prints, per organism and parameter tensor, the count
and max of the differing weights (GPU diagnostic)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist  # noqa: E402
from serann.engine.base import TrainConfig  # noqa: E402
from serann.engine.hip_engine import HipPopulationEngine  # noqa: E402
from serann.genome.interpreter import interpret  # noqa: E402
from tests.archs import ARCHS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--moments", default="16bit")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--n-train", type=int, default=2200)
    ap.add_argument("--archs", default="")
    ap.add_argument("--fuse", default="1,0", help="SERANN_FUSE_ADAM of the two fits")
    a = ap.parse_args()
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=a.n_train, n_test=300, seed=8),
                           n_train=a.n_train, n_test=300)
    names = sorted(ARCHS) if not a.archs else a.archs.split(",")
    irs = [interpret(ARCHS[n]) for n in names]
    cfg = TrainConfig(epochs=a.epochs, batch_size=256, adam_moments=a.moments)
    out = []
    for fuse in a.fuse.split(","):
        os.environ["SERANN_FUSE_ADAM"] = fuse
        eng = HipPopulationEngine(irs, list(range(len(irs))), device="cuda", cfg=cfg)
        eng.fit(data, cfg)
        out.append((eng.p.cpu(), eng.m.cpu().float(), eng.v.cpu().float(), eng.layouts))
        del eng
    (p1, m1, v1, lay), (p0, m0, v0, _) = out
    bad = (p1 != p0) | (m1 != m0) | (v1 != v0)
    print("differing elements:", int(bad.sum()), "of", bad.numel())
    for o, (n, L) in enumerate(zip(names, lay)):
        for kind in ("w", "b", "gamma", "beta"):
            for nid, off in getattr(L, kind).items():
                node = L.ir.node(nid)
                size = int(np.prod(node.attrs.get("wshape", ()))) if kind == "w" and "wshape" in node.attrs else None
                if size is None:
                    size = {"w": int(node.attrs.get("f", 1)) * int(node.attrs.get("cin", 1)) *
                            int(node.attrs.get("kh", 1)) * int(node.attrs.get("kw", 1))}.get(kind, int(node.attrs.get("f", node.shape[-1])))
                seg = bad[off:off + size]
                if seg.any():
                    d = float((p1[off:off + size] - p0[off:off + size]).abs().max())
                    idx = torch.nonzero(seg).flatten()[:6].tolist()
                    print(f"org {o} {n} {kind}[{nid}] {node.attrs.get('kind')} size {size}: {int(seg.sum())} differ,"
                          f" max |dp| {d:.3g}, first {idx}")


if __name__ == "__main__":
    main()
