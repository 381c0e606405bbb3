"""Diagnostic: a fused path (default: Conv2D+MaxPool2D; argv: flag name, arch prefix) vs the unfused HIP path vs the fp32 CPU oracle, per parameter.

Prints the relative Frobenius error of every gradient for the three pairs, so a tolerance failure of
tests/test_gpu_engine.py::test_convpool_fusion_matches_unfused can be attributed (fused kernel wrong,
or bf16 tie-breaking in the unfused pool).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from serann.engine import hip_engine as he  # noqa: E402
from serann.genome.interpreter import interpret  # noqa: E402
from serann.models.organism import init_params  # noqa: E402
from tests.archs import ARCHS  # noqa: E402
from tests.test_gpu_engine import _batch, _oracle, _rel  # noqa: E402


def main():
    flag = sys.argv[1] if len(sys.argv) > 1 else "FUSE_CONVPOOL"
    prefix = sys.argv[2] if len(sys.argv) > 2 else "convpool"
    for name in sorted(ARCHS):
        if not name.startswith(prefix):
            continue
        ir = interpret(ARCHS[name])
        for seed, bseed, B in ((5, 4, 80), (7, 0, 96)):
            params = init_params(ir, seed)
            x, g, y = _batch(B, seed=bseed)
            setattr(he, flag, True)
            fused = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
            gf, _ = fused.debug_train_step(x, g, y)
            setattr(he, flag, False)
            plain = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
            gp, _ = plain.debug_train_step(x, g, y)
            setattr(he, flag, True)
            _, ref = _oracle(ir, params, x, g, y)
            a, b = fused.export_arena(0, gf), plain.export_arena(0, gp)
            for nid in ref:
                for k in ref[nid]:
                    print(f"{name:24s} s{seed} n{nid} {k:8s} fused-oracle {_rel(a[nid][k], ref[nid][k]):.4f} "
                          f"unfused-oracle {_rel(b[nid][k], ref[nid][k]):.4f} fused-unfused {_rel(a[nid][k], b[nid][k]):.4f} "
                          f"|ref| {np.linalg.norm(ref[nid][k]):.3e}",
                          flush=True)


if __name__ == "__main__":
    main()
