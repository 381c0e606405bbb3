#!/usr/bin/env python
"""Per-problem anatomy of the GEMM launches of one training step (measurement helper).

Builds the one-stream train plan of a population file, times every gemm3 launch of the chosen mode in isolation
and prints, per launch: variant, blocks, median time, and per problem its shape (M, N, K, C, KH x KW, H x W), flags,
tiles and the longest k range of a tile (Dense / 1x1 WGRAD: 32-row steps) -- to see whether a launch's time is set
by its block count, by one problem's long tiles, or by padding waste (e.g. C = 1 convolutions).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--population-file", default="populations/bench_gen3_pop125.json")
    ap.add_argument("--batch", type=int, default=750)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--top", type=int, default=14)
    ap.add_argument("--mode", default="wgrad", choices=["fwd", "dgrad", "wgrad"])
    a = ap.parse_args()
    from serann.engine.hip_engine import HipPopulationEngine, Plan
    from serann.genome.interpreter import try_interpret
    from serann.ops import hip_ops as H

    with open(a.population_file) as f:
        irs = [r.ir for r in (try_interpret(s) for s in json.load(f)) if r.ok]
    dev = torch.device("cuda")
    eng = HipPopulationEngine(irs, list(range(len(irs))), device=dev)
    B = a.batch
    mem = eng._alloc_buffers(B, with_grads=True)
    xb = torch.rand(B, 784, device=dev).bfloat16()
    gb = torch.randint(0, 2, (B, 100), device=dev).bfloat16()
    yb = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)
    metrics = torch.zeros(len(irs), 4, dtype=torch.int64, device=dev)
    inputs = [{"X": xb.data_ptr(), "g": gb.data_ptr()} for _ in irs]
    plan = eng._build_plan("train", B, mem, inputs, yb.data_ptr(), [gb.data_ptr()] * len(irs), metrics)
    p = Plan()
    p.launches = plan.launches
    p.run()
    torch.cuda.synchronize()
    out = []
    for i, la in enumerate(plan.launches):
        mode = {"fwd": H.MODE_FWD, "dgrad": H.MODE_DGRAD, "wgrad": H.MODE_WGRAD}[a.mode]
        if la.kind != "gemm3" or la.arg[0] != mode:
            continue
        one = Plan()
        one.launches = [la]
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            one.run()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        d = np.frombuffer(la.descs.cpu().numpy().tobytes(), dtype=H.GEMM_DTYPE)
        t = la.tiles.cpu().numpy().reshape(-1, 4)[:la.n]
        ks = ((t[:, 3] >> 16) & 0xffff) - (t[:, 3] & 0xffff)
        probs = []
        for pi, r in enumerate(d):
            sel = t[:, 0] == pi
            probs.append(dict(M=int(r["M"]), N=int(r["N"]), K=int(r["K"]), C=int(r["C"]), act=int(r["act"]),
                              KH=int(r["KH"]), KW=int(r["KW"]), H=int(r["H"]), W=int(r["W"]),
                              flags=int(r["flags"]), tiles=int(sel.sum()),
                              kmax=int(ks[sel].max()) if sel.any() else 0))
        out.append(dict(i=i, v=int(la.arg[1]), blocks=int(la.n), us=float(np.median(ts)) * 1e6,
                        kmax=int(ks.max()), kmean=float(ks.mean()), probs=probs))
    tot = sum(o["us"] for o in out)
    print(f"{len(out)} {a.mode} launches, {tot / 1e3:.2f} ms isolated")
    for o in sorted(out, key=lambda o: -o["us"])[:a.top]:
        print(f"#{o['i']:3d} v={o['v']} blocks={o['blocks']} {o['us']:7.1f} us  k-steps/tile max {o['kmax']} "
              f"mean {o['kmean']:.1f}")
        for q in sorted(o["probs"], key=lambda q: -q["kmax"] * q["tiles"])[:5]:
            print(f"      M={q['M']:5d} N={q['N']:6d} K={q['K']:7d} C={q['C']:5d} act={q['act']} "
                  f"{q['KH']}x{q['KW']} on {q['H']}x{q['W']} flags={q['flags']:5d} tiles={q['tiles']:5d} kmax={q['kmax']}")
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/{a.mode}_tail.json", "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
