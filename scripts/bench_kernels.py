#!/usr/bin/env python
"""Per-launch timing of one training step of the HIP engine on a generator-sampled population.

Builds the train plan for P organisms, then times every launch individually (median of N
repetitions, synchronised) and attributes time to (kind, mode, variant, problem class), where the
problem class of a GEMM is conv (KH*KW > 1), dense-4d (1x1 with many rows per sample) or dense
(one row per sample: M_Dense / heads).  Prints a table and writes JSON to --out.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=104)
    ap.add_argument("--batch", type=int, default=750)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--out", default="gpurun_out/bench_kernels.json")
    a = ap.parse_args()
    from serann.engine.hip_engine import HipPopulationEngine, Plan
    from serann.genome.codec import decoded_form
    from serann.genome.generator import generate
    from serann.genome.interpreter import try_interpret
    from serann.ops import hip_ops as H

    df = generate(a.pop * 3, seed=a.seed, validation_genotype_size=100)
    irs = []
    for s in df["code"]:
        r = try_interpret(decoded_form(s))
        if r.ok and r.parameters_count <= 2e6:
            irs.append(r.ir)
        if len(irs) == a.pop:
            break
    dev = torch.device("cuda")
    eng = HipPopulationEngine(irs, list(range(len(irs))), device=dev)
    B = a.batch
    mem = eng._alloc_buffers(B, with_grads=True)
    xb = torch.rand(B, 784, device=dev).bfloat16()
    gb = torch.randint(0, 2, (B, 100), device=dev).bfloat16()
    yb = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)
    eng._input_tensors = {xb.data_ptr(): xb, gb.data_ptr(): gb}
    metrics = torch.zeros(len(irs), 4, device=dev)
    inputs = [{"X": xb.data_ptr(), "g": gb.data_ptr()} for _ in irs]
    plan = eng._build_plan("train", B, mem, inputs, yb.data_ptr(), [gb.data_ptr()] * len(irs), metrics)
    # one full step to initialise
    p = Plan()
    p.launches = plan.launches
    p.run()
    torch.cuda.synchronize()
    rows = []
    total_flops = 0.0
    for ir in irs:
        total_flops += 3 * ir.flops_per_sample() * B
    for i, la in enumerate(plan.launches):
        one = Plan()
        one.launches = [la]
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            one.run()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        cls = ""
        if la.kind in ("gemm", "gemm2", "gemm3"):
            d = np.frombuffer(la.descs.cpu().numpy().tobytes(), dtype=H.GEMM_DTYPE)
            kinds = set()
            for r in d:
                if r["KH"] * r["KW"] > 1:
                    kinds.add("conv")
                elif r["H"] * r["W"] > 1 or r["OH"] * r["OW"] > 1:
                    kinds.add("dense4d")
                else:
                    kinds.add("dense")
            cls = "+".join(sorted(kinds))
            mode = la.arg[0] if la.kind in ("gemm2", "gemm3") else la.arg
            flops = float(sum(2.0 * r["M"] * r["N"] * r["K"] for r in d))
        else:
            flops = 0.0
        rows.append(dict(i=i, kind=la.kind, arg=str(la.arg), cls=cls, ms=float(np.median(ts)) * 1e3,
                         tiles=int(la.n), tflops=flops / max(np.median(ts), 1e-9) / 1e12 if flops else 0.0))
    agg = defaultdict(lambda: [0.0, 0])
    for r in rows:
        k = (r["kind"], r["arg"], r["cls"])
        agg[k][0] += r["ms"]
        agg[k][1] += 1
    tot = sum(r["ms"] for r in rows)
    print(f"organisms={len(irs)} launches={len(rows)} step_ms(sum of isolated launches)={tot:.2f} "
          f"train_flops/step={total_flops / 1e12:.3f} TF -> {total_flops / tot / 1e9:.1f} TF/s")
    for k, (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{k[0]:10s} {k[1]:10s} {k[2]:18s} n={n:4d} {ms:9.3f} ms {100 * ms / tot:5.1f}%")
    top = sorted(rows, key=lambda r: -r["ms"])[:15]
    for r in top:
        print(r)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"rows": rows, "total_ms": tot, "train_tflop": total_flops / 1e12}, f)


if __name__ == "__main__":
    main()
