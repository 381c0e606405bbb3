#!/usr/bin/env python
"""Micro-benchmark of the BatchNormalizationF16 kernel phases (achieved HBM bandwidth)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from serann.ops import hip_ops as H


def main():
    dev = "cuda"
    L, s = H.lib(), H.stream_handle()
    for R, C in [(588000, 67), (363000, 64), (96000, 128), (750, 128), (750, 256), (750, 37), (363000, 16)]:
        x = torch.randn(R, C, device=dev).bfloat16()
        y = torch.zeros_like(x); dy = torch.randn_like(x); dx = torch.zeros_like(x)
        f = lambda n: torch.zeros(n, device=dev)
        gamma, beta, mm, mv, mean, invstd, ws, dg, db = f(C) + 1, f(C), f(C), f(C) + 1, f(C), f(C), f(2 * H.BN_WS_STRIPES * C), f(C), f(C)
        row = dict(x=x.data_ptr(), y=y.data_ptr(), dy=dy.data_ptr(), dx=dx.data_ptr(), gamma=gamma.data_ptr(),
                   beta=beta.data_ptr(), mm=mm.data_ptr(), mv=mv.data_ptr(), mean=mean.data_ptr(),
                   invstd=invstd.data_ptr(), ws=ws.data_ptr(), dgamma=dg.data_ptr(), dbeta=db.data_ptr(), R=R, C=C,
                   flags=3, eps=1e-3, momentum=0.99)
        a = np.zeros(1, dtype=H.BN_DTYPE)
        for k, v in row.items():
            a[0][k] = v
        d = torch.as_tensor(np.frombuffer(a.tobytes(), dtype=np.uint8).copy(), device=dev)
        t = torch.as_tensor(H.chunk_tiles([H.bn_chunks(R, C)], 1), device=dev)
        ts = torch.as_tensor(H.chunk_tiles([H.bn_chunks(R, C, stats=True)], 1), device=dev)
        out = []
        for ph, nbytes in [(0, 2), (2, 4), (4, 4), (5, 6)]:
            tt = ts if ph in (0, 4) else t
            for _ in range(3):
                L.bn(ph, d.data_ptr(), tt.data_ptr(), len(tt), s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                L.bn(ph, d.data_ptr(), tt.data_ptr(), len(tt), s)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 20 * 1e3
            out.append(f"ph{ph} {ms:.4f}ms {R * C * nbytes / ms / 1e6:.0f}GB/s")
        print(f"R={R} C={C} tiles={len(t)}: " + "  ".join(out), flush=True)


if __name__ == "__main__":
    main()
