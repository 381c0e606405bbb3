"""RiboAE trainer (reference: ribosomal_autoencoder/training.py:25-133).

Schedules (per batch number b, clamped to the schedule length):
* temperature: logspace(log10(0.3), -3, 5e6)      (computed in closed form, not materialised)
* learning rate: logspace(log10(3e-4), log10(2e-5), 1e6)
* KL weight: linspace(0, 0.2, 1e7) ** 2
Optimizer: Keras Adam (eps 1e-7) with the scheduled learning rate.  Batches are consumed in dataset
order with ``repeat()`` semantics (no shuffle), batch 512.

Engines: on an MI355X the ConcreteGAE step runs on this repository's HIP kernels end to end
(:class:`serann.riboae.hip_trainer.HipRiboTrainer`: gemm3 convolutions / Dense, bn_kernel
BatchNormalization, fused concrete-sample / log-likelihood kernels, the arena Adam; ``engine="hip"``,
the default on a GPU); ``engine="torch"`` keeps the PyTorch reference path (bf16 autocast on a GPU).  Prints every 10 batches, a reconstruction
every 50, and keeps only the most recent best-loss checkpoint at least ``min_backup_interval`` batches
after the previous one -- plus (new) optimizer state + step so training can resume, bf16 autocast on
MI355X, and an optional ``max_steps`` stop condition (the reference loop is infinite).
"""
from __future__ import annotations

import math
import os
import time
from typing import Optional

import numpy as np
import torch

from ..engine.torch_engine import KerasAdam
from ..models.riboae import ConcreteGAE
from .io import save_checkpoint

TEMPERATURE_STEPS = int(5e6)
LEARNING_RATE_STEPS = int(1e6)
KLD_STEPS = int(1e7)


def _logspace_at(start, stop, n, i):
    i = min(i, n - 1)
    return 10 ** (start + (stop - start) * i / (n - 1))


def temperature_at(b):
    return _logspace_at(math.log10(0.3), -3.0, TEMPERATURE_STEPS, b)


def learning_rate_at(b):
    return _logspace_at(math.log10(3e-4), math.log10(2e-5), LEARNING_RATE_STEPS, b)


def kld_weight_at(b):
    b = min(b, KLD_STEPS - 1)
    return (0.2 * b / (KLD_STEPS - 1)) ** 2


class ScheduledKerasAdam(KerasAdam):
    def step(self, lr: Optional[float] = None):
        if lr is not None:
            self.lr = lr
        super().step()

    def state_dict(self):
        return {"t": self.t, "m": [m.detach().cpu() for m in self.m], "v": [v.detach().cpu() for v in self.v]}

    def load_state_dict(self, st):
        """Accepts this optimizer's per-parameter lists (also written by the HIP trainer next to its
        arenas).  Arena-only states from older HIP checkpoints cannot be mapped without the HIP trainer:
        Adam then restarts from t = 0 with zero moments instead of mixing a large t with fresh moments."""
        if "m" not in st or "v" not in st:
            self.t = 0
            for buf in list(self.m) + list(self.v):
                buf.zero_()
            return
        if len(st["m"]) != len(self.m):
            raise ValueError(f"optimizer state has {len(st['m'])} moments, model has {len(self.m)}")
        self.t = int(st["t"])
        with torch.no_grad():
            for dst, src in zip(self.m, st["m"]):
                dst.copy_(src.to(dst.device).reshape(dst.shape))
            for dst, src in zip(self.v, st["v"]):
                dst.copy_(src.to(dst.device).reshape(dst.shape))


def get_dataset(sequences: np.ndarray, train_test_ratio: float):
    split = int(len(sequences) * train_test_ratio)
    return sequences[:split], sequences[split:]


def train(experiment_name: str, model, train_tokens: np.ndarray, vocabulary, out_dir: str, batch_size: int = 512,
          min_backup_interval: int = 1000, max_steps: Optional[int] = None, device="cpu", log=print,
          resume_path: Optional[str] = None, bf16: Optional[bool] = None, demo_every: int = 50, log_every: int = 10,
          engine: str = "auto"):
    dev = torch.device(device)
    model.to(dev).train()
    is_concrete = isinstance(model, ConcreteGAE)
    if engine == "auto":
        engine = "torch"
        if dev.type == "cuda" and is_concrete and os.environ.get("SERANN_RIBOAE_HIP", "1") != "0":
            from ..ops.riboae_ops import available
            if not available():
                raise RuntimeError("serann_hip extension not loadable on a GPU device (build it, or pass engine='torch')")
            engine = "hip"
    hip = None
    start = 1
    min_loss, min_loss_batch = float("inf"), 0
    ck = None
    if resume_path:
        ck = torch.load(resume_path, map_location=dev, weights_only=True)
        model.load_state_dict(ck["state_dict"])
        start = int(ck["step"]) + 1
        min_loss = float(ck.get("extra", {}).get("loss", min_loss))
        min_loss_batch = int(ck["step"])
    if engine == "hip":
        from .hip_trainer import HipRiboTrainer
        hip = HipRiboTrainer(model, device=dev, eps=1e-7)      # re-points the parameters into its arenas
        opt = hip                                               # checkpoints carry its Adam state
    else:
        opt = ScheduledKerasAdam(list(model.parameters()), lr=learning_rate_at(1), eps=1e-7)
    if ck is not None and ck.get("optimizer"):
        opt.load_state_dict(ck["optimizer"])                    # either engine reads either format
    if bf16 is None:
        bf16 = dev.type == "cuda"
    # the token dataset lives on the device for the HIP engine (int32, the kernels' token type): a batch is a view,
    # not a host slice + upload per step
    data = torch.as_tensor(np.asarray(train_tokens), dtype=torch.long)
    if hip is not None:
        data = data.to(dev, torch.int32)
    n = len(data)
    nb = max(1, math.ceil(n / batch_size))
    history = []
    b = start
    t0 = time.perf_counter()
    # The step's loss is read back one step late (HIP engine): the host enqueues step b before it waits for step
    # b - 1's loss, so the GPU does not idle on the host between steps.  A backup of step b - 1 must hold step b - 1's
    # weights, so while b - 1 is far enough from the last backup to be backed up, its loss is read (and the backup
    # taken) before step b is enqueued; the decisions are the reference's (training.py:92-101), step for step.
    pending = None                     # (step, metrics) whose loss has not been read yet

    def settle(step_, metrics_):
        nonlocal min_loss, min_loss_batch, t0
        loss_ = float(metrics_["loss"].detach())
        history.append(loss_)
        if step_ % log_every == 0:
            log(f'Batch: {step_} | Loss: {loss_:.5f} | NLL: {float(metrics_["nll"].detach()):.5f} | '
                f'KL: {float(metrics_["kld"].detach()):.5f} '
                f'| {(time.perf_counter() - t0) / log_every * 1e3:.1f} ms/batch')
            t0 = time.perf_counter()
        return loss_

    def backup(step_, loss_):
        nonlocal min_loss, min_loss_batch
        path = os.path.join(out_dir, f"{experiment_name}_b{step_}.pt")
        log("Backing up to: ", path)
        save_checkpoint(path, model, "concrete" if is_concrete else "deterministic", step_, opt.state_dict(),
                        {"loss": loss_})
        prev = os.path.join(out_dir, f"{experiment_name}_b{min_loss_batch}.pt")
        if min_loss_batch > 0 and os.path.exists(prev) and prev != path:
            os.remove(prev)
        min_loss, min_loss_batch = loss_, step_

    while max_steps is None or b < start + max_steps:
        i = (b - 1) % nb
        x = data[i * batch_size:(i + 1) * batch_size]
        if x.device != dev:
            x = x.to(dev, non_blocking=True)
        temperature, lr, kw = temperature_at(b), learning_rate_at(b), kld_weight_at(b)
        if hip is not None:
            # a backup of step b - 1 must see step b - 1's weights: when b - 1 may be backed up (its distance to
            # the last backup allows it), its loss is settled before step b is enqueued
            if pending is not None and pending[0] - min_loss_batch >= min_backup_interval:
                loss = settle(*pending)
                if loss < min_loss:
                    backup(pending[0], loss)
                pending = None
            metrics = hip.step(x, temperature, kw, lr)
            if pending is not None:
                settle(*pending)        # (b - 1 could not be backed up: reading its loss now costs nothing)
            pending = (b, metrics)
        else:
            with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=bool(bf16)):
                metrics = model.compute_loss(x, temperature, kw) if is_concrete else model.compute_loss(x)
            opt.zero_grad()
            metrics["loss"].float().backward()
            opt.step(lr)
            loss = settle(b, metrics)
            if loss < min_loss and b - min_loss_batch >= min_backup_interval:
                backup(b, loss)
        model._param_version = getattr(model, "_param_version", 0) + 1
        if vocabulary is not None and demo_every and b % demo_every == 0:
            model.eval()
            with torch.no_grad():
                z = model.encode(x[:1].long())
                seq = model.decode(z).cpu().numpy()
            model.train()
            log(f"\n\nOriginal: \n{vocabulary.decode(x[:1].cpu().numpy())[0]}\n\n")
            log(f"Genotype:\n{''.join(str(int(v)) for v in z[0].cpu().numpy())}\n\n")
            log(f"Reconstruction: \n{vocabulary.decode(seq)[0]}\n\n")
        b += 1
    if pending is not None:
        loss = settle(*pending)
        if loss < min_loss and pending[0] - min_loss_batch >= min_backup_interval:
            backup(pending[0], loss)
    if max_steps is not None and b - 1 != min_loss_batch:
        # bounded runs always leave a final checkpoint (the reference loop never ends)
        path = os.path.join(out_dir, f"{experiment_name}_b{b - 1}.pt")
        save_checkpoint(path, model, "concrete" if is_concrete else "deterministic", b - 1, opt.state_dict(),
                        {"loss": history[-1] if history else float("nan"), "final": True})
        log("Final checkpoint: ", path)
    return history
