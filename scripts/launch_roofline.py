#!/usr/bin/env python
"""Per-launch roofline of the single-stream training step: the kernel trace of a ``--streams 1`` bench_step
run aligned launch by launch with the same plan rebuilt on the CPU (as scripts/launch_table.py), and for
every launch a lower bound on its time from the problems in its descriptor table:

    ideal = max(minimum bytes / HBM_BW, model FLOPs / MFMA_PEAK)

where minimum bytes count every operand read once and every output written once (weights, activations,
Q40 gradients; the fused-Adam epilogue's p / m / v / bf16 copy), and FLOPs are the GEMM's 2 M N K.  The
table is sorted by the gap (measured - ideal): where the step's time goes beyond what the work requires.

    python scripts/launch_roofline.py gpurun_out/tl/kernel_trace.csv --population-file populations/bench_gen3_pop125.json
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

HBM = 5.0e12        # B/s, achievable streaming rate used for the bound (MI355X: 6.3 measured copy, 8 spec)
PEAK = 2.5e15       # bf16 dense MFMA


def _rows(la, dtype):
    raw = la.descs.cpu().numpy().tobytes()
    return np.frombuffer(raw, dtype=dtype)


def gemm_cost(mode, r):
    """(bytes, flops) of one gemm3 problem from its descriptor record."""
    from serann.ops import hip_ops as H
    M, N, K = int(r["M"]), int(r["N"]), int(r["K"])
    flags = int(r["flags"])
    fl = 2.0 * M * N * K
    if mode == H.MODE_FWD:
        a = (M // max(1, int(r["OH"]) * int(r["OW"]))) * int(r["H"]) * int(r["W"]) * int(r["C"]) * 2
        out = M * N * (4 if flags & H.GF_OUT_F32 else 2)
        if flags & H.GF_SPLITWS:
            out = M * N * 4                                   # fp32 partial slab of this split
        return a + N * K * 2 + out, fl
    if mode == H.MODE_DGRAD:
        rows = M // max(1, int(r["H"]) * int(r["W"]))         # batch
        dz = rows * int(r["OH"]) * int(r["OW"]) * int(r["F"]) * 2
        y = dz if int(r["act"]) else 0
        # GF_NBNSUM: no dY store, fp32 per-column BN sums per 128-row m tile instead
        out = -(-M // 128) * N * H.NBN_NSUM * 4 if flags & H.GF_NBNSUM else M * N * 2
        return dz + y + N * K * 2 + out, fl
    # WGRAD: M = F, N = KH KW C, K = rows
    rows = K // max(1, int(r["OH"]) * int(r["OW"]))
    dz = K * int(r["F"]) * 2
    y = dz if int(r["act"]) else 0
    x = rows * int(r["H"]) * int(r["W"]) * int(r["C"]) * 2
    if flags & H.GF_ADAM:
        out = M * N * 26                                      # p, m, v read + written, bf16 copy written
    else:
        out = M * N * 8                                       # Q40 gradient (one writer or atomics)
    return dz + y + x + out, fl


def launch_cost(la, B):
    from serann.ops import hip_ops as H
    k = la.kind
    if k == "gemm3":
        mode = la.arg[0]
        b = f = 0.0
        for r in _rows(la, H.GEMM_DTYPE):
            bb, ff = gemm_cost(mode, r)
            b += bb
            f += ff
        return b, f
    if k == "bn":
        rows = _rows(la, H.BN_DTYPE)
        n = float(sum(int(r["R"]) * int(r["C"]) for r in rows))
        phase = la.arg
        per = {0: 2, 2: 4, 3: 4, 4: 4, 5: 6}[phase]           # bytes per element (bf16 in / out)
        return n * per, 0.0
    if k == "pool":
        rows = _rows(la, H.POOL_DTYPE)
        n = float(sum(int(r["B"]) * int(r["H"]) * int(r["W"]) * int(r["C"]) for r in rows))
        return n * (2 + 1) if la.arg == 0 else n * 2 * 2, 0.0
    if k == "copy":
        rows = _rows(la, H.COPY_DTYPE)
        return float(sum(int(r["rows"]) * int(r["cols"]) * 4 for r in rows)), 0.0
    if k == "ew":
        rows = _rows(la, H.EW_DTYPE)
        return float(sum(int(np.prod(r["D"])) * int(np.prod(r["R"])) * 2 + int(np.prod(r["D"])) * 2 for r in rows)), 0.0
    if k == "splitfin":
        rows = _rows(la, H.SPLITFIN_DTYPE)
        return float(sum(int(r["M"]) * int(r["N"]) * (4 * int(r["S"]) + 2) for r in rows)), 0.0
    if k == "convpool":
        rows = _rows(la, H.CONVPOOL_DTYPE)
        b = f = 0.0
        for r in rows:
            img = int(r["B"]) * int(r["H"]) * int(r["W"]) * 2
            pooled = int(r["B"]) * int(r["POH"]) * int(r["POW"]) * int(r["F"]) * 3
            b += img + pooled
            f += 2.0 * int(r["B"]) * int(r["OH"]) * int(r["OW"]) * int(r["F"]) * int(r["KH"]) * int(r["KW"])
        return b, f
    if k == "nbn" and la.arg[0] == 6:
        rows = _rows(la, H.NBN_DTYPE)                          # phase 6: read the DGRAD's partial sums
        return float(sum(int(r["mtiles"]) * int(r["np"]) * int(r["F"]) * H.NBN_NSUM * 4 for r in rows)), 0.0
    if k == "nbn":
        rows = _rows(la, H.NBN_DTYPE)
        b = f = 0.0
        for r in rows:
            b += int(r["R"]) * (int(r["K"]) * 2 + int(r["F"]) * 2)
            f += 2.0 * int(r["R"]) * int(r["F"]) * int(r["K"])
        return b, f
    if k == "gchain":
        rows = _rows(la, H.GCHAIN_DTYPE)
        b = f = 0.0
        for r in rows:
            b += int(r["B"]) * (int(r["L0"]) * 2 + int(r["L1"]) * int(r["F2"]) * 2)
            f += 2.0 * int(r["B"]) * int(r["L1"]) * (int(r["F1"]) * int(r["T"]) + int(r["F1"]) * int(r["F2"]))
        return b, f
    if k in ("transpose", "imcol"):
        return 0.0, 0.0
    return 0.0, 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--population-file", default="populations/bench_gen3_pop125.json")
    ap.add_argument("--pop", type=int, default=125)
    ap.add_argument("--batch", type=int, default=750)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--params-per-step-adam", action="store_true")
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
    wall = statistics.median((s[-1][1] - s[0][0]) / 1e3 for s in steps)

    from serann.engine.hip_engine import HipPopulationEngine
    from serann.genome.interpreter import try_interpret
    with open(a.population_file) as f:
        irs = [try_interpret(s).ir for s in json.load(f)][:a.pop]
    eng = HipPopulationEngine(irs, list(range(len(irs))), device="cpu")
    mem = eng._alloc_buffers(a.batch, with_grads=True)
    pl = eng._build_plan("train", a.batch, mem, [{"X": 0, "g": 0} for _ in irs], 0, [0] * len(irs), None,
                         adam_ctx=1)
    launches = pl.launches
    fwd = pl.fwd_count
    order = [("pre", None)] * 3 + [("plan", la) for la in launches[:fwd]] + [("loss", None)] + \
            [("plan", la) for la in launches[fwd:]] + [("post", None)] * 2
    if len(order) != n_common:
        print(f"warning: trace step has {n_common} kernels, plan gives {len(order)}; alignment is approximate")
    rows = []
    for i in range(min(len(order), n_common)):
        d = statistics.median((s[i][1] - s[i][0]) / 1e3 for s in steps)
        kind, la = order[i]
        b, f = launch_cost(la, a.batch) if la is not None else (0.0, 0.0)
        if kind == "post" and i == len(order) - 2:
            b = float(eng.p.numel()) * (4 * 3 + 8 + 2 + 4 * 3) * 0.0     # arena pass: measured separately
        ideal = max(b / HBM, f / PEAK) * 1e6
        rows.append(dict(i=i, kernel=steps[0][i][2], kind=la.kind if la else kind, arg=str(la.arg) if la else "",
                         blocks=la.n if la else None, us=d, ideal_us=ideal, gb=b / 1e9, gflop=f / 1e9))
    total = sum(r["us"] for r in rows)
    ideal = sum(r["ideal_us"] for r in rows)
    print(f"{len(steps)} steps, {n_common} kernels/step; wall {wall / 1e3:.2f} ms/step, kernel sum {total / 1e3:.2f} ms, "
          f"ideal sum {ideal / 1e3:.2f} ms ({sum(r['gb'] for r in rows):.2f} GB, {sum(r['gflop'] for r in rows):.0f} GFLOP)")
    by = defaultdict(lambda: [0.0, 0.0, 0])
    for r in rows:
        fam = re.sub(r"<.*", "", r["kernel"])
        by[fam][0] += r["us"]
        by[fam][1] += r["ideal_us"]
        by[fam][2] += 1
    print(f"\n{'family':<34s} {'launches':>8s} {'ms':>7s} {'ideal ms':>9s} {'x ideal':>8s}")
    for fam, (us, idl, n) in sorted(by.items(), key=lambda kv: -(kv[1][0] - kv[1][1])):
        print(f"{fam[:34]:<34s} {n:8d} {us / 1e3:7.2f} {idl / 1e3:9.2f} {us / max(idl, 1e-9):8.1f}")
    print(f"\n{'#':>4s} {'us':>8s} {'ideal':>8s} {'gap':>8s} {'GB':>6s} {'GFLOP':>7s} {'blocks':>7s}  kernel")
    for r in sorted(rows, key=lambda r: -(r["us"] - r["ideal_us"]))[:a.top]:
        print(f"{r['i']:4d} {r['us']:8.1f} {r['ideal_us']:8.1f} {r['us'] - r['ideal_us']:8.1f} {r['gb']:6.3f} "
              f"{r['gflop']:7.1f} {str(r['blocks']):>7s}  {r['kernel'][:56]} {r['arg']}")


if __name__ == "__main__":
    main()
