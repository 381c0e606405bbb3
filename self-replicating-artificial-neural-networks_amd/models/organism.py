"""Torch oracle organism: an ``nn.Module`` built from :class:`OrganismIR` with Keras-2.6 semantics.

This is the reference-semantics path (SURVEY §7.1 ``eager.py``): it runs on CPU (tests, the
pop=2 plumbing config) and GPU, and is the numerics oracle for the HIP grouped engine.

Semantics reproduced (reference citations):
* glorot-uniform kernels, zero biases, BN gamma=1 beta=0 moving mean 0 / variance 1 (Keras defaults,
  SURVEY §2.7);
* BatchNormalizationF16 (common/BatchNormalizationF16.py:81-153): training normalises with the
  biased batch variance, the moving variance is updated with the factor n/(n-(1+eps)), moving
  averages use ``x <- x*momentum + value*(1-momentum)``; inference uses moving statistics;
* heads Dense(C)->softmax and Dense(L)->sigmoid on ``Reshape((1,-1))(con)`` (common/logic.py:29-33).
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ..genome.ir import Node, OrganismIR


def glorot_limit(node: Node) -> float:
    a = node.attrs
    rf = a["kh"] * a["kw"]
    return math.sqrt(6.0 / (rf * a["cin"] + rf * a["f"]))


def init_params(ir: OrganismIR, seed: int) -> Dict[int, Dict[str, np.ndarray]]:
    """Deterministic Keras-default initialisation keyed by node id (float32 numpy)."""
    rng = np.random.default_rng(seed)
    out: Dict[int, Dict[str, np.ndarray]] = {}
    for n in ir.nodes:
        p = {}
        if n.op == "gemm":
            lim = glorot_limit(n)
            a = n.attrs
            p["kernel"] = rng.uniform(-lim, lim, size=(a["kh"], a["kw"], a["cin"], a["f"])).astype(np.float32)
            if a["use_bias"]:
                p["bias"] = np.zeros((a["f"],), np.float32)
        elif n.op == "bn":
            c = n.attrs["channels"]
            if n.attrs["scale"]:
                p["gamma"] = np.ones((c,), np.float32)
            if n.attrs["center"]:
                p["beta"] = np.zeros((c,), np.float32)
            p["moving_mean"] = np.zeros((c,), np.float32)
            p["moving_variance"] = np.ones((c,), np.float32)
        if p:
            out[n.id] = p
    return out


def _act(x: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return torch.relu(x)
    if act == "sigmoid":
        return torch.sigmoid(x)
    return x


class Organism(torch.nn.Module):
    def __init__(self, ir: OrganismIR, params: Dict[int, Dict[str, np.ndarray]],
                 device="cpu", dtype=torch.float32):
        super().__init__()
        self.ir = ir
        self.params = torch.nn.ParameterDict()
        self.bufs: Dict[str, torch.Tensor] = {}
        for nid, p in params.items():
            for k, v in p.items():
                t = torch.as_tensor(v, device=device, dtype=torch.float32)
                if k.startswith("moving_"):
                    self.register_buffer(f"n{nid}_{k}", t.clone())
                else:
                    self.params[f"n{nid}_{k}"] = torch.nn.Parameter(t.clone())
        self.compute_dtype = dtype

    def p(self, nid: int, name: str):
        key = f"n{nid}_{name}"
        if key in self.params:
            return self.params[key]
        return getattr(self, key, None)

    def forward(self, x: torch.Tensor, g: torch.Tensor, training: bool) -> Tuple[torch.Tensor, torch.Tensor]:
        """x: (B, H, W, 1), g: (B, L, 1).  Returns (class logits (B, C), replication logits (B, L))."""
        ir = self.ir
        B = x.shape[0]
        vals: Dict[int, torch.Tensor] = {}
        for n in ir.nodes:
            if n.op == "input":
                vals[n.id] = x if n.attrs["name"] == "X" else g
                continue
            ins = [vals[i] for i in n.inputs]
            if n.op == "gemm":
                vals[n.id] = self._gemm(n, ins[0], B)
            elif n.op == "pool":
                a = n.attrs
                t = ins[0].permute(0, 3, 1, 2)
                t = F.max_pool2d(t, (a["ph"], a["pw"]), (a["sh"], a["sw"]))
                vals[n.id] = t.permute(0, 2, 3, 1).contiguous()
            elif n.op == "bn":
                vals[n.id] = self._bn(n, ins[0], training)
            elif n.op == "reshape":
                vals[n.id] = ins[0].reshape((B,) + n.shape)
            elif n.op == "concat":
                vals[n.id] = torch.cat(ins, dim=n.attrs["axis"])
            elif n.op == "neg":
                vals[n.id] = -ins[0]
            elif n.op == "sub":
                m = n.attrs["mode"]
                if m == "tt":
                    vals[n.id] = ins[0] - ins[1]
                elif m == "tc":
                    vals[n.id] = ins[0] - n.attrs["c"]
                else:
                    vals[n.id] = n.attrs["c"] - ins[0]
            else:
                raise ValueError(n.op)
        return vals[ir.cls_head].reshape(B, -1), vals[ir.rep_head].reshape(B, -1)

    def _gemm(self, n: Node, x: torch.Tensor, B: int) -> torch.Tensor:
        a = n.attrs
        w = self.p(n.id, "kernel")
        b = self.p(n.id, "bias") if a["use_bias"] else None
        dt = self.compute_dtype
        if a["kh"] == 1 and a["kw"] == 1 and a["sh"] == 1 and a["sw"] == 1:
            y = x.reshape(B, -1, a["cin"]).to(dt) @ w.reshape(a["cin"], a["f"]).to(dt)
            y = y.float()
            if b is not None:
                y = y + b
        else:
            t = x.reshape(B, a["h"], a["w"], a["cin"]).permute(0, 3, 1, 2).to(dt)
            wt = w.permute(3, 2, 0, 1).to(dt)
            y = F.conv2d(t, wt, None, (a["sh"], a["sw"])).float()
            if b is not None:
                y = y + b.view(1, -1, 1, 1)
            y = y.permute(0, 2, 3, 1)
        return _act(y, a["act"]).reshape((B,) + n.shape)

    def _bn(self, n: Node, x: torch.Tensor, training: bool) -> torch.Tensor:
        a = n.attrs
        ax = a["axis"]
        red = [d for d in range(x.dim()) if d != ax]
        bshape = [1] * x.dim()
        bshape[ax] = a["channels"]
        gamma = self.p(n.id, "gamma")
        beta = self.p(n.id, "beta")
        mm = self.p(n.id, "moving_mean")
        mv = self.p(n.id, "moving_variance")
        eps = a["epsilon"]
        if training:
            mean = x.mean(dim=red)
            var = x.var(dim=red, unbiased=False)
            y = (x - mean.view(bshape)) / torch.sqrt(var.view(bshape) + eps)
            with torch.no_grad():
                nsamp = float(np.prod([x.shape[d] for d in red]))
                mom = a["momentum"]
                unbiased = var.detach() * (nsamp / (nsamp - (1.0 + eps)))
                mm.mul_(mom).add_(mean.detach() * (1 - mom))
                mv.mul_(mom).add_(unbiased * (1 - mom))
        else:
            y = (x - mm.view(bshape)) / torch.sqrt(mv.view(bshape) + eps)
        if gamma is not None:
            y = y * gamma.view(bshape)
        if beta is not None:
            y = y + beta.view(bshape)
        return y
