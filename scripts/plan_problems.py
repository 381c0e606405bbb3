#!/usr/bin/env python
"""Problem shapes of selected launches of the single-stream training plan (CPU only; nothing is launched).

Launch indices are the step-kernel positions printed by scripts/launch_table.py (a step is gather, memset,
adam_scalars, the forward launches, the loss, the backward launches, adam, counter), so a slow row of that
table can be looked up here:

    python scripts/plan_problems.py 202 180 273 [--population-file populations/bench_gen3_pop125.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("index", nargs="+", type=int)
    ap.add_argument("--population-file", default="populations/bench_gen3_pop125.json")
    ap.add_argument("--pop", type=int, default=125)
    ap.add_argument("--batch", type=int, default=750)
    a = ap.parse_args()
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.genome.interpreter import try_interpret
    from serann.ops import hip_ops as H

    with open(a.population_file) as f:
        irs = [try_interpret(s).ir for s in json.load(f)][:a.pop]
    eng = HipPopulationEngine(irs, list(range(len(irs))), device="cpu")
    mem = eng._alloc_buffers(a.batch, with_grads=True)
    pl = eng._build_plan("train", a.batch, mem, [{"X": 0, "g": 0} for _ in irs], 0, [0] * len(irs), None,
                         adam_ctx=1)
    launches = [la for la in pl.launches if la.kind != "fn"]
    order = [None] * 3 + launches[:pl.fwd_count] + [None] + launches[pl.fwd_count:]
    for i in a.index:
        la = order[i] if 0 <= i < len(order) else None
        if la is None or la.kind != "gemm3":
            print(i, "not a gemm3 launch:", la.kind if la is not None else "step prologue / loss / epilogue")
            continue
        d = np.frombuffer(la.descs.numpy().tobytes(), dtype=H.GEMM_DTYPE)
        shapes = Counter((int(r["M"]), int(r["N"]), int(r["K"]), int(r["KH"]), int(r["KW"]), int(r["C"]),
                          int(r["flags"])) for r in d)
        print(i, la.arg, la.n, "blocks", len(d), "problems")
        for k, v in shapes.most_common(12):
            print("   M,N,K,KH,KW,C,flags", k, "x", v)


if __name__ == "__main__":
    main()
