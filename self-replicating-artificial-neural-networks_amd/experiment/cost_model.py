"""Per-organism training-time model used to balance organisms across ranks (LPT, parallel/partition.py).

Replaces the reference's round-robin job split (evolutionary_experiment/logic/experiment.py:170-178)
and the round-2 FLOP count + constant.  A rank trains its shard as ONE grouped engine, so its step time
is additive over organisms in three measurable per-organism features plus a shard constant:

    t_step(shard) ~= sum_k coef_k * sum_organisms feature_k + d

over the features of :func:`features` (conv / dense FLOPs, BatchNorm / other activation elements, nodes).  The coefficients are fitted by non-negative least squares to measured replay
times of random sub-populations on one MI355X (scripts/calibrate_cost.py) and stored in
``parameters/cost_model.json``; without that file a roofline default is used (100 TFLOP/s effective
MFMA rate, 1.5 TB/s effective bandwidth, 2 us per node).
"""
from __future__ import annotations

import json
import math
from functools import lru_cache
from pathlib import Path
from typing import Dict, Sequence

MODEL_FILE = Path(__file__).resolve().parent.parent / "parameters" / "cost_model.json"
DEFAULT = {"a_s_per_flop": 1.0 / 100e12, "b_s_per_byte": 1.0 / 1.5e12, "c_s_per_node": 2e-6, "d_s": 0.0,
           "source": "roofline default (no calibration file)"}


PER_SAMPLE = ("Fc", "Fd", "Ab", "Aa")        # features that scale with the batch (times 3 for FLOPs: fwd + 2 bwd)


def features(ir) -> Dict[str, float]:
    """Per-organism features.  Round-3 set (fitted by scripts/calibrate_cost.py): Fc / Fd = forward FLOPs per
    sample of convolutions (KH*KW > 1) / of Dense, 1x1 and head GEMMs (MFMA work at different
    efficiencies), Ab / Aa = activation elements per sample of BatchNormalization tensors (several
    streaming passes each) / of every other node's inputs and output, N = compute nodes.  The round-2
    aggregate (F, A, N) is kept for coefficient files that use it."""
    by_id = {n.id: n for n in ir.nodes}
    out = dict(F=0.0, A=0.0, N=0.0, Fc=0.0, Fd=0.0, Ab=0.0, Aa=0.0)
    for n in ir.nodes:
        if n.op in ("input", "reshape"):
            continue
        elems = float(math.prod(n.shape)) + sum(float(math.prod(by_id[i].shape)) for i in n.inputs)
        f = n.flops_per_sample()
        out["F"] += f
        out["A"] += 6.0 * 2.0 * elems
        out["N"] += 1.0
        if n.op == "gemm" and n.attrs.get("kh", 1) * n.attrs.get("kw", 1) > 1:
            out["Fc"] += f
        else:
            out["Fd"] += f
        out["Ab" if n.op == "bn" else "Aa"] += elems
    return out


@lru_cache(maxsize=4)
def _load(path: str) -> dict:
    p = Path(path)
    if p.exists():
        with open(p) as f:
            return {**DEFAULT, **json.load(f)}
    return dict(DEFAULT)


def coefficients(path: Path = MODEL_FILE) -> dict:
    return _load(str(path))


def organism_time(ir, batch: int = 750, coef: dict = None) -> float:
    """Predicted seconds per training step this organism adds to its shard (at ``batch`` rows)."""
    c = coef or coefficients()
    f = features(ir)
    if "coef" in c:                  # named-feature fit (Fc, Fd, Ab, Aa, N)
        t = 0.0
        for k, v in c["coef"].items():
            scale = (3.0 * batch if k.startswith("F") else float(batch)) if k in PER_SAMPLE else 1.0
            t += v * f[k] * scale
        return t
    return (c["a_s_per_flop"] * 3.0 * f["F"] * batch + c["b_s_per_byte"] * f["A"] * batch
            + c["c_s_per_node"] * f["N"])


def shard_time(irs: Sequence, batch: int = 750, coef: dict = None) -> float:
    c = coef or coefficients()
    return sum(organism_time(ir, batch, c) for ir in irs) + (c["d_s"] if len(irs) else 0.0)
