#!/usr/bin/env python
"""BASELINE config #3: ribosomal-autoencoder training (bf16 autocast) on one MI355X, synthetic dataset.

Reports training batches/s and sequences/s (batch 512, ConcreteGAE, schedules of training.py), plus
the HIP decode path throughput (genotypes decoded per second; BN folded, grouped MFMA GEMM + fused
group-argmax) and its agreement with the torch eval-mode decode.
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
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--decode-n", type=int, default=4096)
    a = ap.parse_args()
    from serann.genome.generator import generate
    from serann.genome.tokenizer import Vocabulary, tokenize
    from serann.models.riboae import ConcreteGAE
    from serann.riboae.trainer import train

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    df = generate(2048, seed=0)
    vocab = Vocabulary.build(tokenize(s) for s in df["code"])
    seqs = vocab.encode_strings(list(df["code"]), 350)
    model = ConcreteGAE(100, 350, len(vocab), 50, 2, prior_temperature=0.01)
    quiet = lambda *x, **k: None  # noqa: E731
    train("bench", model, seqs, None, "/tmp/serann_riboae_bench", batch_size=a.batch, min_backup_interval=10 ** 9,
          max_steps=a.warmup, device=dev, log=quiet, demo_every=0)
    if dev == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    hist = train("bench", model, seqs, None, "/tmp/serann_riboae_bench", batch_size=a.batch,
                 min_backup_interval=10 ** 9, max_steps=a.steps, device=dev, log=quiet, demo_every=0)
    if dev == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"metric": "riboae_train_sequences_per_sec", "value": a.steps * a.batch / dt, "batches_per_sec": a.steps / dt,
           "ms_per_batch": dt / a.steps * 1e3, "batch": a.batch, "dtype": "bf16 autocast", "loss_first": hist[0],
           "loss_last": hist[-1], "device": dev, "params": sum(p.numel() for p in model.parameters())}
    g = np.random.default_rng(0).integers(0, 2, (a.decode_n, 100))
    model.eval()
    ref = model.decode(torch.as_tensor(g, device=dev)).cpu().numpy()
    model.decode_tokens(g[:8], device=dev)
    if dev == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = model.decode_tokens(g, device=dev)
    if dev == "cuda":
        torch.cuda.synchronize()
    out["decode_genotypes_per_sec"] = a.decode_n / (time.perf_counter() - t0)
    out["decode_token_agreement_vs_torch"] = float((got == ref).mean())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
