"""Per-organism training-time model used to balance organisms across ranks (LPT, parallel/partition.py).

Replaces the reference's round-robin job split (evolutionary_experiment/logic/experiment.py:170-178)
and the round-2 FLOP count + constant.  A rank trains its shard as ONE grouped engine, so its step time
is additive over organisms in three measurable per-organism features plus a shard constant:

    t_step(shard) ~= a * sum F + b * sum A + c * sum N + d

F = forward FLOPs per sample (MFMA work), A = activation bytes per sample that the forward + backward
passes stream (memory work), N = layer nodes (per-node launch / latency share inside the grouped
launches of a level).  The coefficients are fitted by non-negative least squares to measured replay
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


def features(ir) -> Dict[str, float]:
    """(F, A, N) of one organism: forward FLOPs / sample, streamed activation bytes / sample (6 bf16
    passes over every node's inputs and output across forward + backward), and compute nodes."""
    by_id = {n.id: n for n in ir.nodes}
    F = A = N = 0.0
    for n in ir.nodes:
        if n.op in ("input", "reshape"):
            continue
        elems = float(math.prod(n.shape)) + sum(float(math.prod(by_id[i].shape)) for i in n.inputs)
        F += n.flops_per_sample()
        A += 6.0 * 2.0 * elems
        N += 1.0
    return {"F": F, "A": A, "N": N}


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
    return (c["a_s_per_flop"] * 3.0 * f["F"] * batch + c["b_s_per_byte"] * f["A"] * batch
            + c["c_s_per_node"] * f["N"])


def shard_time(irs: Sequence, batch: int = 750, coef: dict = None) -> float:
    c = coef or coefficients()
    return sum(organism_time(ir, batch, c) for ir in irs) + (c["d_s"] if len(irs) else 0.0)
