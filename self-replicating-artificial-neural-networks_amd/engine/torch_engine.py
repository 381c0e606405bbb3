"""Torch oracle population engine (reference-semantics path; CPU and GPU).

Each organism is an :class:`~serann.models.organism.Organism`; one joint loss, one Keras-Adam over
all parameters -- exactly the reference's fused ``Model`` + ``fit`` structure
(experiment_worker.py:66-83) -- but organisms never see each other's rows during replication.
"""
from __future__ import annotations

import time
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..genome.ir import OrganismIR
from ..models.organism import Organism, init_params
from .base import FitResult, PopulationEngine, TrainConfig, epoch_permutation


class KerasAdam:
    """TF ``ResourceApplyAdam`` update: lr_t = lr*sqrt(1-b2^t)/(1-b1^t);
    p -= lr_t * m / (sqrt(v) + eps)  (eps outside the bias correction, unlike torch.optim.Adam)."""

    def __init__(self, params: Sequence[torch.Tensor], lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-4):
        self.params = [p for p in params]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.t = 0

    @torch.no_grad()
    def step(self):
        self.t += 1
        lr_t = self.lr * (1 - self.b2 ** self.t) ** 0.5 / (1 - self.b1 ** self.t)
        ps = [p for p in self.params if p.grad is not None]
        if not ps:
            return
        idx = [i for i, p in enumerate(self.params) if p.grad is not None]
        gs = [self.params[i].grad for i in idx]
        ms = [self.m[i] for i in idx]
        vs = [self.v[i] for i in idx]
        torch._foreach_mul_(ms, self.b1)
        torch._foreach_add_(ms, gs, alpha=1 - self.b1)
        torch._foreach_mul_(vs, self.b2)
        torch._foreach_addcmul_(vs, gs, gs, value=1 - self.b2)
        denom = torch._foreach_sqrt(vs)
        torch._foreach_add_(denom, self.eps)
        torch._foreach_addcdiv_(ps, ms, denom, value=-lr_t)

    def zero_grad(self):
        for p in self.params:
            p.grad = None


class TorchPopulationEngine(PopulationEngine):
    def __init__(self, irs: Sequence[OrganismIR], seeds: Sequence[int], device="cpu",
                 compute_dtype=torch.float32, cfg: Optional[TrainConfig] = None):
        self.device = torch.device(device)
        self.irs = list(irs)
        self.cfg = cfg or TrainConfig()
        self.orgs: List[Organism] = [Organism(ir, init_params(ir, s), self.device, compute_dtype)
                                     for ir, s in zip(self.irs, seeds)]
        self.num_organisms = len(self.orgs)
        self.lb = torch.tensor([ir.loss_balance for ir in self.irs], dtype=torch.float32, device=self.device)
        params = [p for o in self.orgs for p in o.parameters()]
        c = self.cfg
        self.opt = KerasAdam(params, c.lr, c.beta1, c.beta2, c.eps)

    # ------------------------------------------------------------------------------------------
    def _to(self, a, dtype=torch.float32):
        return torch.as_tensor(np.ascontiguousarray(a), device=self.device, dtype=dtype)

    def fit(self, data, cfg: Optional[TrainConfig] = None) -> FitResult:
        cfg = cfg or self.cfg
        P = self.num_organisms
        X = self._to(data.train_x)
        Y = self._to(data.train_labels, torch.long)
        G = self._to(data.train_g)
        n = len(X)
        split = cfg.split(n)
        steps = cfg.steps_per_epoch(split)
        t0 = time.perf_counter()
        train_acc = np.zeros(P)
        val_acc = np.full(P, np.nan)
        val_mse = np.full(P, np.nan)
        total_steps = 0
        for epoch in range(cfg.epochs):
            perm = torch.as_tensor(epoch_permutation(cfg.seed, epoch, split), device=self.device)
            correct = torch.zeros(P, device=self.device)
            seen = 0
            for s in range(steps):
                idx = perm[s * cfg.batch_size:(s + 1) * cfg.batch_size]
                xb, yb, gb = X[idx], Y[idx], G[idx]
                loss = 0.0
                for i, org in enumerate(self.orgs):
                    cl, rl = org(xb, gb[..., None], training=True)
                    ce = F.cross_entropy(cl, yb)
                    mse = ((torch.sigmoid(rl) - gb) ** 2).mean()
                    loss = loss + self.lb[i] * ce + (1 - self.lb[i]) * mse
                    correct[i] += (cl.argmax(1) == yb).sum()
                self.opt.zero_grad()
                loss.backward()
                self.opt.step()
                seen += len(idx)
                total_steps += 1
            train_acc = (correct / max(seen, 1)).cpu().numpy()
            if cfg.val_every_epoch or epoch == cfg.epochs - 1:
                val_acc, val_mse = self._eval(X[split:], Y[split:], G[split:], cfg)
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        return FitResult(train_acc, val_acc, val_mse, time.perf_counter() - t0, total_steps)

    @torch.no_grad()
    def _eval(self, X, Y, G, cfg):
        P = self.num_organisms
        if len(X) == 0:
            return np.full(P, np.nan), np.full(P, np.nan)
        correct = torch.zeros(P, device=self.device, dtype=torch.float64)
        sq = torch.zeros(P, device=self.device, dtype=torch.float64)
        for s in range(0, len(X), cfg.eval_batch):
            xb, yb, gb = X[s:s + cfg.eval_batch], Y[s:s + cfg.eval_batch], G[s:s + cfg.eval_batch]
            for i, org in enumerate(self.orgs):
                cl, rl = org(xb, gb[..., None], training=False)
                correct[i] += (cl.argmax(1) == yb).sum()
                sq[i] += ((torch.sigmoid(rl) - gb) ** 2).mean(1).sum()
        n = len(X)
        return (correct / n).cpu().numpy(), (sq / n).cpu().numpy()

    def evaluate(self, x, labels, g, cfg: Optional[TrainConfig] = None) -> np.ndarray:
        cfg = cfg or self.cfg
        acc, _ = self._eval(self._to(x), self._to(labels, torch.long), self._to(g), cfg)
        return acc

    @torch.no_grad()
    def replicate(self, genotypes, images, cfg: Optional[TrainConfig] = None) -> List[np.ndarray]:
        out = []
        for i, org in enumerate(self.orgs):
            pool = len(images[i])
            xb = self._to(images[i])
            gb = self._to(np.repeat(np.asarray(genotypes[i], np.float32)[None], pool, 0))
            _, rl = org(xb, gb[..., None], training=False)
            # Keras predicts in float16: round the sigmoid output through fp16
            out.append(torch.sigmoid(rl).half().float().cpu().numpy())
        return out
