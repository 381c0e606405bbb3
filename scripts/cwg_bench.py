#!/usr/bin/env python
"""Isolated timing of the conv WGRAD kernel (gemm3.hip g3_conv_wgrad_kernel) and its split finalize on
single problems of the bench's generation-3 population (or --shape B,H,W,C,F,K,S): median of --reps
launches each, TFLOP/s of the GEMM and slab bytes.  Planner knobs come from the environment (SERANN_CONV_*).

    python scripts/cwg_bench.py [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

SHAPES = [  # B, H, W, C, F, K, S (generation-3 bench population, heaviest first)
    (750, 28, 28, 74, 16, 5, 1),
    (750, 24, 24, 32, 16, 5, 1),
    (750, 28, 28, 64, 16, 5, 1),
    (750, 14, 14, 61, 64, 5, 1),
    (750, 24, 24, 32, 16, 7, 1),
    (750, 24, 24, 8, 16, 7, 1),
    (750, 20, 20, 16, 16, 3, 1),
    (750, 12, 12, 64, 64, 3, 1),
    (750, 100, 1, 80, 64, 3, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shape", action="append", default=None)
    a = ap.parse_args()
    from serann.ops import hip_ops as H
    L = H.lib()
    dev = "cuda"
    shapes = [tuple(int(v) for v in s.split(",")) for s in a.shape] if a.shape else SHAPES
    for B, Hh, Ww, C, F, K, S in shapes:
        KW = K if Ww > 1 else 1
        OH, OW = (Hh - K) // S + 1, (Ww - KW) // S + 1
        x = H.padded(torch.randn(B, Hh, Ww, C, device=dev).bfloat16())
        dz = H.padded(torch.randn(B, OH, OW, F, device=dev).bfloat16())
        dw = H.padded(torch.zeros(F * K * KW * C, dtype=torch.int64, device=dev))
        row = dict(a=dz.data_ptr(), b=x.data_ptr(), out=dw.data_ptr(), H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=F, KH=K,
                   KW=KW, SH=S, SW=S, M=F, N=K * KW * C, K=B * OH * OW, flags=0)
        plans = H.gemm3_plan(H.MODE_WGRAD, [row], [(F, K * KW * C, B * OH * OW)])
        keep, runs = [], []
        for v, rws, tiles in plans:
            fin = []
            for r in rws:
                if r.get("_wgfin"):
                    ws = torch.empty(H.wgrad_slab_elems(r) + 64, dtype=torch.float32, device=dev)
                    keep.append(ws)
                    fin.append(H.wgrad_finalize_row(r, ws.data_ptr()))
            rec = H.record_array([{k: val for k, val in r.items() if not k.startswith("_")} for r in rws], H.GEMM_DTYPE)
            H.fill_gemm_divisors(rec)
            d = torch.as_tensor(np.frombuffer(rec.tobytes(), np.uint8).copy(), device=dev)
            t = torch.as_tensor(tiles, device=dev)
            keep += [d, t]
            runs.append(("gemm", lambda v=v, d=d, t=t: L.gemm3(H.MODE_WGRAD, v, d.data_ptr(), t.data_ptr(), len(t),
                                                               H.stream_handle()), v, len(t)))
            if fin:
                fr = H.record_array(fin, H.WGFIN_DTYPE)
                fd = torch.as_tensor(np.frombuffer(fr.tobytes(), np.uint8).copy(), device=dev)
                ft = torch.as_tensor(H.chunk_tiles([f["M"] * f["N"] for f in fin], H.WGFIN_ELEMS), device=dev)
                keep += [fd, ft]
                runs.append(("fin", lambda fd=fd, ft=ft: L.wgrad_finalize(fd.data_ptr(), ft.data_ptr(), len(ft),
                                                                        H.stream_handle()), fin[0]["S"], len(ft)))
        torch.cuda.synchronize()
        flop = 2.0 * F * K * KW * C * B * OH * OW
        line = [f"B{B} {Hh}x{Ww}x{C} F{F} k{K}x{KW} s{S}: {flop / 1e9:.1f} GF"]
        for name, fn, info, nblk in runs:
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            us = statistics.median(ts)
            extra = f" {flop / us / 1e6:.0f} TF/s" if name == "gemm" else f" S={info}"
            line.append(f"{name}[{info} x{nblk}] {us:.1f} us{extra}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
