#!/usr/bin/env python
"""Per-launch table of the single-stream training step: the kernel trace of a ``--streams 1`` bench_step
run (scripts/gpu_timeline.sh with STREAMS=1) aligned, launch by launch, with the same plan rebuilt on the
CPU (scripts/plan_grid.py), so every launch gets its median duration over the steps, its block count and
its problems.  Sorted by time; the launch-order index lets a row be found in the plan.

    python scripts/launch_table.py gpurun_out/tl/kernel_trace.csv --population-file populations/bench_gen3_pop125.json
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--population-file", default="populations/bench_gen3_pop125.json")
    ap.add_argument("--pop", type=int, default=125)
    ap.add_argument("--batch", type=int, default=750)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out", default=None, help="write the full table as JSON")
    a = ap.parse_args()
    ev = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       re.sub(r"\(.*$", "", r["Kernel_Name"].replace("void ", ""))))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[2].startswith("gather_batch")]
    steps = [ev[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    n_common = statistics.mode(len(s) for s in steps)
    steps = [s for s in steps if len(s) == n_common]

    from serann.engine.hip_engine import HipPopulationEngine
    from serann.genome.interpreter import try_interpret
    from serann.ops import hip_ops as H
    with open(a.population_file) as f:
        irs = [try_interpret(s).ir for s in json.load(f)][:a.pop]
    eng = HipPopulationEngine(irs, list(range(len(irs))), device="cpu")
    mem = eng._alloc_buffers(a.batch, with_grads=True)
    pl = eng._build_plan("train", a.batch, mem, [{"X": 0, "g": 0} for _ in irs], 0, [0] * len(irs), None,
                         adam_ctx=0)
    launches = [la for la in pl.launches if la.kind != "fn"]
    # step = gather, memset, adam_scalars, fwd launches, loss, bwd launches, adam, counter
    fwd = pl.fwd_count
    order = [("pre", None)] * 3 + [("plan", la) for la in launches[:fwd]] + [("loss", None)] + \
            [("plan", la) for la in launches[fwd:]] + [("post", None)] * 2
    if len(order) != n_common:
        print(f"warning: trace step has {n_common} kernels, plan gives {len(order)}; alignment is approximate")
    rows = []
    total = 0.0
    for i in range(min(len(order), n_common)):
        d = statistics.median((s[i][1] - s[i][0]) / 1e3 for s in steps)
        total += d
        kind, la = order[i]
        nprob = None
        if la is not None and la.kind == "gemm3":
            nprob = int(la.descs.numel() * la.descs.element_size()) // H.GEMM_DTYPE.itemsize
        rows.append({"i": i, "kernel": steps[0][i][2], "kind": la.kind if la else kind,
                     "arg": str(la.arg) if la else "", "blocks": la.n if la else None, "problems": nprob, "us": d})
    print(f"{len(steps)} steps, {n_common} kernels per step, median kernel time per step {total / 1e3:.2f} ms")
    print(f"{'#':>4s} {'us':>8s} {'cum%':>6s} {'blocks':>7s} {'probs':>6s}  kernel")
    cum = 0.0
    for r in sorted(rows, key=lambda r: -r["us"])[:a.top]:
        cum += r["us"]
        print(f"{r['i']:4d} {r['us']:8.1f} {100 * cum / total:6.1f} {str(r['blocks']):>7s} {str(r['problems']):>6s}  "
              f"{r['kernel'][:60]} {r['arg']}")
    small = [r for r in rows if r["blocks"] is not None and r["blocks"] < 256]
    print(f"launches with < 256 blocks: {len(small)}, {sum(r['us'] for r in small) / 1e3:.2f} ms per step")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=0)


if __name__ == "__main__":
    main()
