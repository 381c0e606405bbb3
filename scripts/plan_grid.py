#!/usr/bin/env python
"""Grid sizes of the training plan (runs on the CPU: the plan is built against host buffers, nothing is
launched).  For every launch of the single-stream train plan: kind, instantiation, blocks and problems;
then a histogram of launches by block count -- a launch with fewer blocks than the chip has CUs (256)
cannot fill it, whatever its kernel does.

    python scripts/plan_grid.py --population-file populations/bench_gen3_pop125.json [--streams 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--population-file", default="populations/bench_gen3_pop125.json")
    ap.add_argument("--pop", type=int, default=125)
    ap.add_argument("--batch", type=int, default=750)
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--kind", default=None, help="only launches of this kind (e.g. gemm3)")
    a = ap.parse_args()
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.genome.interpreter import try_interpret

    with open(a.population_file) as f:
        irs = [try_interpret(s).ir for s in json.load(f)][:a.pop]
    eng = HipPopulationEngine(irs, list(range(len(irs))), device="cpu")
    mem = eng._alloc_buffers(a.batch, with_grads=True)
    inputs = [{"X": 0, "g": 0} for _ in irs]
    hist = Counter()
    for grp in eng._stream_groups(a.streams):
        pl = eng._build_plan("train", a.batch, mem, inputs, 0, [0] * len(irs), None, orgs=grp, adam_ctx=0)
        for i, la in enumerate(pl.launches):
            if a.kind and la.kind != a.kind:
                continue
            nprob = int(la.descs.shape[0]) if la.descs is not None and la.descs.dim() > 0 else 0
            tag = "fwd" if i < pl.fwd_count else "bwd"
            print(f"{tag} {la.kind:9s} {str(la.arg):18s} blocks={la.n:6d} problems={nprob}")
            b = la.n
            hist["<64" if b < 64 else "64-255" if b < 256 else "256-1023" if b < 1024 else ">=1024"] += 1
    print("launches by blocks:", dict(hist))


if __name__ == "__main__":
    main()
