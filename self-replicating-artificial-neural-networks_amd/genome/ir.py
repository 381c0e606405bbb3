"""Layer IR for SeRANN organisms.

An organism is a small DAG over two inputs -- the image ``X`` of shape (H, W, 1) and the genotype
``g`` of shape (L, 1) -- ending in two heads attached to ``Reshape((1, -1))(con)``
(reference: common/logic.py:17-35).  All shapes in the IR exclude the batch dimension.

Every trainable op is lowered to one of a handful of *engine kinds* so that the population engine
can batch heterogeneous organisms into grouped kernels:

* ``gemm``   -- Dense on the last axis, Conv2D, Conv1D, and the heads are all NHWC implicit-GEMM
                convolutions ``(H, W, C) --(KH, KW, SH, SW)--> (OH, OW, F)`` (+ bias, + act);
* ``pool``   -- MaxPool2D (valid);
* ``bn``     -- BatchNormalizationF16 (batch statistics in training, moving statistics otherwise);
* ``reshape``-- a view (activations are contiguous row-major, so it is free);
* ``concat`` -- copy into column slices;
* ``ewise``  -- rare elementwise ops reachable by mutation (``-x``, ``x - y`` with broadcasting).
"""
from __future__ import annotations

import hashlib
import os
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

Shape = Tuple[int, ...]

ACTIVATIONS = ("linear", "relu", "sigmoid")


@dataclass
class Node:
    id: int
    op: str                      # input | gemm | pool | bn | reshape | concat | neg | sub
    inputs: List[int]
    shape: Shape                 # output shape (no batch)
    attrs: Dict = field(default_factory=dict)

    # ---- parameter bookkeeping -------------------------------------------------------------
    def param_shapes(self) -> Dict[str, Shape]:
        a = self.attrs
        if self.op == "gemm":
            shapes = {"kernel": (a["kh"], a["kw"], a["cin"], a["f"])}
            if a["use_bias"]:
                shapes["bias"] = (a["f"],)
            return shapes
        if self.op == "bn":
            c = a["channels"]
            shapes = {}
            if a["scale"]:
                shapes["gamma"] = (c,)
            if a["center"]:
                shapes["beta"] = (c,)
            return shapes
        return {}

    def buffer_shapes(self) -> Dict[str, Shape]:
        if self.op == "bn":
            c = self.attrs["channels"]
            return {"moving_mean": (c,), "moving_variance": (c,)}
        return {}

    def num_params(self) -> int:
        """Keras ``count_params`` contribution (trainable + non-trainable weights)."""
        n = sum(math.prod(s) for s in self.param_shapes().values())
        n += sum(math.prod(s) for s in self.buffer_shapes().values())
        return n

    def flops_per_sample(self) -> float:
        """Forward FLOPs per sample (multiply-add = 2)."""
        a = self.attrs
        if self.op == "gemm":
            oh, ow = a["oh"], a["ow"]
            return 2.0 * a["rows"] * oh * ow * a["kh"] * a["kw"] * a["cin"] * a["f"]
        if self.op in ("bn", "pool", "neg", "sub", "concat"):
            return float(math.prod(self.shape)) * (4 if self.op == "bn" else 1)
        return 0.0

    def signature(self) -> str:
        items = ",".join(f"{k}={self.attrs[k]}" for k in sorted(self.attrs) if k != "source")
        return f"{self.op}({items})<-{self.inputs}:{self.shape}"


@dataclass
class OrganismIR:
    """Interpreted organism: the reachable DAG plus the two heads."""
    nodes: List[Node]            # topologically ordered; nodes[0] = X input, nodes[1] = g input
    con: int                     # node id of ``con``
    loss_balance: float
    num_classes: int
    genotype_size: int
    head_features: int           # D = prod(con.shape)

    # head nodes (classification Dense(C) + replication Dense(L)) are appended as gemm nodes
    cls_head: int = -1
    rep_head: int = -1

    def node(self, i: int) -> Node:
        return self.by_id[i]

    def __post_init__(self):
        self.by_id = {n.id: n for n in self.nodes}

    @property
    def trainable_nodes(self) -> List[Node]:
        return [n for n in self.nodes if n.param_shapes()]

    def count_params(self) -> int:
        return sum(n.num_params() for n in self.nodes)

    def flops_per_sample(self) -> float:
        return sum(n.flops_per_sample() for n in self.nodes)

    def cost_per_sample(self) -> float:
        """Estimated training time per sample (arbitrary units) of this organism on the HIP engine: per
        node the larger of its MFMA time and its memory time (a roofline with the rates the grouped
        kernels reach on small layers, measured: ~100 TFLOP/s, ~1.5 TB/s), summed over forward +
        backward (3x the forward FLOPs; ~6 passes over each node's input and output, bf16).  Used to
        balance organisms across ranks and HIP streams: FLOPs alone under-weight the memory-bound
        layers (BatchNormalization, Dense on 75,000-row inputs) that dominate many organisms."""
        if os.environ.get("SERANN_COST", "time") == "flops":
            return 3.0 * self.flops_per_sample()
        by_id = {n.id: n for n in self.nodes}
        t = 0.0
        for n in self.nodes:
            if n.op in ("input", "reshape"):
                continue
            elems = float(math.prod(n.shape)) + sum(float(math.prod(by_id[i].shape)) for i in n.inputs)
            t += max(3.0 * n.flops_per_sample() / 100e12, 6.0 * 2.0 * elems / 1.5e12)
        return t * 1e12

    def activation_elems_per_sample(self) -> int:
        return sum(math.prod(n.shape) for n in self.nodes if n.op not in ("reshape", "input"))

    def arch_hash(self) -> str:
        """Hash of the architecture (topology + shapes + attrs), independent of loss_balance."""
        h = hashlib.md5()
        for n in self.nodes:
            h.update(n.signature().encode())
        return h.hexdigest()

    def consumers(self) -> Dict[int, List[int]]:
        out: Dict[int, List[int]] = {n.id: [] for n in self.nodes}
        for n in self.nodes:
            for i in n.inputs:
                out[i].append(n.id)
        return out


def conv_out(size: int, k: int, s: int) -> int:
    """Keras ``conv_output_length`` with 'valid' padding and dilation 1."""
    return (size - k + s) // s if size - k + 1 > 0 else size - k + 1
