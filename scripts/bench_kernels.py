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


def launch_bytes(la, H):
    """Minimum HBM bytes a launch must move (each operand read once, output written once) and a short
    shape list of its problems."""
    if la.descs is None:
        return 0.0, []
    raw = la.descs.cpu().numpy().tobytes()
    tot, probs = 0.0, []
    if la.kind == "gemm3":
        mode = la.arg[0] if isinstance(la.arg, tuple) else la.arg
        for r in np.frombuffer(raw, dtype=H.GEMM_DTYPE):
            M, N, K = int(r["M"]), int(r["N"]), int(r["K"])
            ob = 4 if int(r["flags"]) & H.GF_OUT_F32 else 2
            if mode == H.MODE_WGRAD:
                ohw = max(1, int(r["OH"]) * int(r["OW"]))
                nb = K // ohw
                b = K * M * 2 + nb * int(r["H"]) * int(r["W"]) * int(r["C"]) * 2 + M * N * 4
            elif mode == H.MODE_FWD:
                ohw = max(1, int(r["OH"]) * int(r["OW"]))
                nb = M // ohw
                b = nb * int(r["H"]) * int(r["W"]) * int(r["C"]) * 2 + N * K * 2 + M * N * ob
            else:
                b = M * N * 2 + N * K * 2 + M * K * 2 // max(1, int(r["KH"]) * int(r["KW"]))
            tot += b
            probs.append((M, N, K, int(r["KH"]), int(r["KW"]), int(r["C"])))
    elif la.kind == "bn":
        for r in np.frombuffer(raw, dtype=H.BN_DTYPE):
            e = int(r["R"]) * int(r["C"])
            tot += e * 2 * {0: 1, 2: 2, 3: 2, 4: 2, 5: 3}.get(int(la.arg), 2)
            probs.append((int(r["R"]), int(r["C"])))
    elif la.kind == "pool":
        for r in np.frombuffer(raw, dtype=H.POOL_DTYPE):
            e_in = int(r["B"]) * int(r["H"]) * int(r["W"]) * int(r["C"])
            e_out = int(r["B"]) * int(r["OH"]) * int(r["OW"]) * int(r["C"])
            tot += e_in * 2 + e_out * 3
            probs.append((int(r["B"]), int(r["H"]), int(r["W"]), int(r["C"])))
    elif la.kind == "copy":
        for r in np.frombuffer(raw, dtype=H.COPY_DTYPE):
            tot += int(r["rows"]) * int(r["cols"]) * 4
            probs.append((int(r["rows"]), int(r["cols"])))
    return tot, probs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=104)
    ap.add_argument("--batch", type=int, default=750)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--out", default="gpurun_out/bench_kernels.json")
    ap.add_argument("--only", type=str, default="", help="comma-separated launch indices to time (profiling)")
    ap.add_argument("--population-file", default=None, help="JSON list of source codes (bench.py --dump-population)")
    ap.add_argument("--ancestor-frac", type=float, default=0.0,
                    help="fraction of clones of the example.json ancestor (table codec): the bench's regime")
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
    if a.population_file:
        with open(a.population_file) as f:
            irs = [try_interpret(s).ir for s in json.load(f)][:a.pop]
    if a.ancestor_frac > 0:
        from serann.config import default_parameters
        from serann.experiment.runner import build_codec
        params = default_parameters("example")
        codec = build_codec(params, "table", seed=0)
        anc = try_interpret(codec.decode_to_string(np.asarray(params["ancestor_genotype"])[None])[0]).ir
        k = int(round(a.ancestor_frac * a.pop))
        irs = [anc] * k + irs[:a.pop - k]
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
    # one full step to initialise
    p = Plan()
    p.launches = plan.launches
    p.run()
    torch.cuda.synchronize()
    rows = []
    total_flops = 0.0
    for ir in irs:
        total_flops += 3 * ir.flops_per_sample() * B
    only = {int(v) for v in a.only.split(",") if v.strip()}
    for i, la in enumerate(plan.launches):
        if only and i not in only:
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
        cls = ""
        nbytes, probs = launch_bytes(la, H)
        if la.kind == "gemm3":
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
            mode = la.arg[0]
            flops = float(sum(2.0 * r["M"] * r["N"] * r["K"] for r in d))
        else:
            flops = 0.0
        med = float(np.median(ts))
        rows.append(dict(i=i, kind=la.kind, arg=str(la.arg), cls=cls, ms=med * 1e3,
                         tiles=int(la.n), tflops=flops / max(med, 1e-9) / 1e12 if flops else 0.0,
                         mbytes=nbytes / 1e6, gbps=nbytes / max(med, 1e-9) / 1e9, probs=probs[:6]))
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
    tb = sum(r["mbytes"] for r in rows)
    print(f"min bytes/step {tb:.1f} MB -> {tb / tot:.1f} GB/s effective over the sum of launches")
    top = sorted(rows, key=lambda r: -r["ms"])[:40]
    for r in top:
        print(f"#{r['i']:3d} {r['kind']:8s} {r['arg']:14s} {r['cls']:16s} {r['ms']:7.3f} ms tiles={r['tiles']:6d} "
              f"{r['tflops']:6.1f} TF/s {r['mbytes']:8.1f} MB {r['gbps']:7.0f} GB/s {r['probs'][:3]}")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"rows": rows, "total_ms": tot, "train_tflop": total_flops / 1e12}, f)


if __name__ == "__main__":
    main()
