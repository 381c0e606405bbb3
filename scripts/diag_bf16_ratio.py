"""Margin of tests/test_gpu_engine.py's bf16-relative criterion per architecture, batch and seed: for every
parameter gradient, a_h / (1.5 a_b + 0.01 |v| + floor) -- a_h / a_b the HIP engine's / PyTorch bf16's error
against the CPU fp32 oracle.  Values < 1 pass.  Run with SERANN_FUSE_GCHAIN=0 (and other fusion switches) to
see whether a fused path is the outlier."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from serann.engine.hip_engine import HipPopulationEngine  # noqa: E402
from serann.genome.interpreter import interpret  # noqa: E402
from serann.models.organism import init_params  # noqa: E402
from tests.archs import ARCHS  # noqa: E402
from tests.test_gpu_engine import _batch, _oracle, _oracle_dev  # noqa: E402

names = sys.argv[1:] or sorted(ARCHS)
for B in (96, 750):
    for name in names:
        ir = interpret(ARCHS[name])
        params = init_params(ir, 7)
        worst = []
        for seed in (0, 1, 2):
            x, g, y = _batch(B, seed=seed)
            eng = HipPopulationEngine([ir], [0], device="cuda", params=[params])
            grads, _ = eng.debug_train_step(x, g, y)
            _, ref = _oracle(ir, params, x, g, y)
            bf = _oracle_dev(ir, params, x, g, y, "cuda", torch.bfloat16)
            hip = eng.export_arena(0, grads)
            eng.close()
            gmax = max(float(np.abs(v).max()) for d in ref.values() for v in d.values())
            m, arg = 0.0, None
            for nid, d in ref.items():
                for k, v in d.items():
                    a_h = np.linalg.norm(np.asarray(hip[nid][k], np.float64) - v)
                    a_b = np.linalg.norm(np.asarray(bf[nid][k], np.float64) - v)
                    floor = 1e-3 * gmax * np.sqrt(v.size)
                    if k == "bias" and "kernel" in d:
                        floor = max(floor, 0.02 * np.linalg.norm(d["kernel"]))
                    r = a_h / (1.5 * a_b + 0.01 * np.linalg.norm(v) + floor)
                    rel_h = a_h / max(np.linalg.norm(v), 1e-30)
                    rel_b = a_b / max(np.linalg.norm(v), 1e-30)
                    if r > m:
                        m, arg = r, (nid, k, round(rel_h, 4), round(rel_b, 4))
            worst.append((round(m, 3), arg))
        print(f"B={B} {name:34s} " + "  ".join(f"{w[0]} {w[1]}" for w in worst), flush=True)
