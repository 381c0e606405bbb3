"""Gradient / logit error of the HIP engine against the CPU fp32 oracle per test architecture, at the
test batch (96) and the production batch (750): the numbers behind tests/test_gpu_engine.py tolerances."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

from serann.engine.hip_engine import HipPopulationEngine  # noqa: E402
from serann.genome.interpreter import interpret  # noqa: E402
from serann.models.organism import init_params  # noqa: E402
from tests.archs import ARCHS  # noqa: E402
from tests.test_gpu_engine import _batch, _oracle, _rel  # noqa: E402

for B in (96, 750):
    worst = []
    for name in sorted(ARCHS):
        ir = interpret(ARCHS[name])
        params = init_params(ir, 7)
        x, g, y = _batch(B)
        eng = HipPopulationEngine([ir], [0], device="cuda", params=[params])
        grads, _ = eng.debug_train_step(x, g, y)
        rl, rg = _oracle(ir, params, x, g, y)
        hg = eng.export_arena(0, grads)
        errs = []
        for nid, d in rg.items():
            for k, v in d.items():
                if np.linalg.norm(v) < 1e-5:
                    continue
                scale = 0.02 * np.linalg.norm(d["kernel"]) if "kernel" in d else 0.0
                got = np.asarray(hg[nid][k], np.float64)
                err = np.linalg.norm(got - v) / max(np.linalg.norm(v), scale, 1e-12)
                cos = float(np.dot(got.ravel(), v.ravel()) / (np.linalg.norm(got) * np.linalg.norm(v) + 1e-30))
                errs.append((err, cos, nid, k))
        e = max(errs)
        c = min(errs, key=lambda t: t[1])
        print(f"B={B} {name:34s} logits {_rel(eng.debug_logits()[0], rl):.4f}  max grad err {e[0]:.4f} ({e[2]},{e[3]})"
              f"  min cos {c[1]:.5f} ({c[2]},{c[3]})", flush=True)
        worst.append(e[0])
        del eng
    print(f"B={B}: worst grad err {max(worst):.4f}", flush=True)
