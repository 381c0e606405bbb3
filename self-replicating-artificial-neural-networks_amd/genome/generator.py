"""Synthetic SeRANN generator (reference: synthetic_serann_generator/generator.py,
synthetic_serann_generator/layer_transitions.py).

The generator reproduces the *distribution* of the reference Markov-chain grammar:

* 13 layer states; the transition probabilities below are the *effective* ones of the reference's
  ``_sample`` (probabilities sorted ascending, first cumulative sum above U ~ U(0,1)).  This matters
  for the ``g`` row, whose entries sum to 1.1: the effective distribution is
  Dense 0.4, Conv1D 0.4, Concatenate 0.2 (layer_transitions.py:16; generator.py:25-30);
* per-layer argument samplers (truncated/clipped normals, power-of-two filters, odd kernels);
* the same source templates (with spaces; the decoded form used by the experiment has none);
* ``loss_balance ~ U(0, 1)`` with 4 decimals; md5 de-duplication; nets that fail to build are
  rejected (the reference validates with genotype length 350 and a linear replication head,
  SURVEY §2.9 item 7 -- ``validation_genotype_size`` reproduces that).

Generation is seeded (the reference seeds from ``os.urandom`` and is not reproducible).
Parameter counting uses the genome interpreter (no TensorFlow).
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Optional, Tuple

import numpy as np

from .interpreter import try_interpret

STATES = ["X", "X_Dense", "X_MaxPool2D", "X_Conv2D", "X_BatchNorm",
          "g", "g_Dense", "g_Conv1D", "g_BatchNorm",
          "M_Concatenate", "M_Dense", "M_BatchNorm", "outputs"]

# effective transition distributions: state -> [(next_state, probability)]
TRANSITIONS: Dict[str, List[Tuple[str, float]]] = {
    "X": [("X_Dense", 0.1), ("X_MaxPool2D", 0.1), ("X_Conv2D", 0.6), ("M_Concatenate", 0.2)],
    "X_Dense": [("X_Dense", 0.1), ("X_Conv2D", 0.2), ("X_BatchNorm", 0.2), ("M_Concatenate", 0.5)],
    "X_MaxPool2D": [("X_Dense", 0.3), ("X_Conv2D", 0.4), ("M_Concatenate", 0.3)],
    "X_Conv2D": [("X_Dense", 0.1), ("X_MaxPool2D", 0.4), ("X_Conv2D", 0.2), ("X_BatchNorm", 0.2),
                 ("M_Concatenate", 0.1)],
    "X_BatchNorm": [("X_Dense", 0.2), ("X_MaxPool2D", 0.1), ("M_Concatenate", 0.7)],
    "g": [("g_Dense", 0.4), ("g_Conv1D", 0.4), ("M_Concatenate", 0.2)],
    "g_Dense": [("g_Dense", 0.1), ("g_Conv1D", 0.2), ("g_BatchNorm", 0.2), ("M_Concatenate", 0.5)],
    "g_Conv1D": [("g_Dense", 0.3), ("g_Conv1D", 0.2), ("g_BatchNorm", 0.2), ("M_Concatenate", 0.3)],
    "g_BatchNorm": [("g_Dense", 0.2), ("g_Conv1D", 0.15), ("M_Concatenate", 0.65)],
    "M_Concatenate": [("M_Dense", 1.0)],
    "M_Dense": [("M_Dense", 0.2), ("M_BatchNorm", 0.2), ("outputs", 0.6)],
    "M_BatchNorm": [("M_Dense", 0.1), ("outputs", 0.9)],
}

TEMPLATES = {
    "X_Dense": "{name} = Dense(units={units}, activation='{activation}')({source})",
    "X_MaxPool2D": "{name} = MaxPool2D(pool_size={pool_size})({source})",
    "X_Conv2D": "{name} = Conv2D(filters={filters}, kernel_size={kernel_size}, strides={strides})({source})",
    "X_BatchNorm": "{name} = BatchNormalization()({source})",
    "g_Dense": "{name} = Dense(units={units}, activation='{activation}')({source})",
    "g_Conv1D": "{name} = Conv1D(filters={filters}, kernel_size={kernel_size}, strides={strides})({source})",
    "g_BatchNorm": "{name} = BatchNormalization()({source})",
    "M_Concatenate": "{name} = concatenate([Reshape((1, -1))({source1}), Reshape((1, -1))({source2})])",
    "M_Dense": "{name} = Dense(units={units}, activation='{activation}')({source})",
    "M_BatchNorm": "{name} = BatchNormalization()({source})",
}


def _clipped_normal(rng: np.random.Generator, mean: float, std: float, lo: int, hi: int) -> int:
    # int() truncates toward zero, then clip (layer_transitions.py:32,36,39,45,49,56)
    return int(np.clip(int(rng.standard_normal() * std + mean), lo, hi))


def _odd_kernel(rng: np.random.Generator) -> int:
    x = int(np.clip(int(rng.standard_normal() * 1.3 + 6), 2, 10))
    return x + (x % 2) - 1


def _choice(rng: np.random.Generator, options: List[Tuple[object, float]]):
    u = rng.random()
    acc = 0.0
    for value, p in options:
        acc += p
        if u < acc:
            return value
    return options[-1][0]


def sample_args(state: str, rng: np.random.Generator) -> Dict[str, object]:
    act = [("relu", 0.8), ("sigmoid", 0.2)]
    if state == "X_Dense":
        return {"units": _clipped_normal(rng, 64, 8, 8, 128), "activation": _choice(rng, act)}
    if state == "g_Dense":
        return {"units": _clipped_normal(rng, 64, 15, 8, 128), "activation": _choice(rng, act)}
    if state == "M_Dense":
        return {"units": _clipped_normal(rng, 128, 30, 32, 256), "activation": _choice(rng, act)}
    if state == "X_MaxPool2D":
        return {"pool_size": _clipped_normal(rng, 2, 1.1, 2, 5)}
    if state in ("X_Conv2D", "g_Conv1D"):
        return {"filters": 2 ** _clipped_normal(rng, 4.5, 1.0, 0, 6), "kernel_size": _odd_kernel(rng),
                "strides": _choice(rng, [(1, 0.8), (2, 0.2)])}
    return {}


def _walk(rng, start_state: str, var: str, stop: str) -> List[str]:
    lines = []
    state = start_state
    while True:
        state = _choice(rng, TRANSITIONS[state])
        if state == stop:
            return lines
        args = dict(name=var, source=var, **sample_args(state, rng))
        lines.append(TEMPLATES[state].format(**args))


def generate_source(rng: np.random.Generator) -> Dict[str, object]:
    """Sample one SeRANN (unvalidated).  Returns the source and branch statistics."""
    x_lines = _walk(rng, "X", "X_layer", "M_Concatenate")
    g_lines = _walk(rng, "g", "g_layer", "M_Concatenate")
    concat = TEMPLATES["M_Concatenate"].format(name="con", source1="X_layer", source2="g_layer")
    m_lines = _walk(rng, "M_Concatenate", "con", "outputs")
    x_branch, g_branch, merged = "\n".join(x_lines), "\n".join(g_lines), "\n".join(m_lines)
    net = "\n\n".join([x_branch, g_branch, concat, merged])
    net_hash = hashlib.md5(net.encode()).hexdigest()
    loss_balance = float(rng.random())
    net += "\n\nloss_balance = {:.4f}".format(loss_balance)
    return {"code": net, "net_hash": net_hash, "last_layer": "con",
            # the reference counts '' as one line (generator.py:94-96)
            "x_layers": len(x_branch.split("\n")), "g_layers": len(g_branch.split("\n")),
            "m_layers": len(merged.split("\n")), "loss_balance": loss_balance}


def generate_network(rng: np.random.Generator, validation_genotype_size: int = 350,
                     image_shape=(28, 28)) -> Optional[Dict[str, object]]:
    """One generator draw; ``None`` when the net fails to build (generator.py:73-99)."""
    rec = generate_source(rng)
    res = try_interpret(rec["code"], image_shape=image_shape, genotype_size=validation_genotype_size)
    if not res.ok:
        return None
    rec["parameters_count"] = int(res.parameters_count)
    return rec


def generate(n: int, seed: int = 0, validation_genotype_size: int = 350, workers: int = 0,
             max_rounds: int = 100):
    """Generate ``n`` unique valid nets (md5 de-dup), as a pandas DataFrame with the reference's
    CSV columns ``code, parameters_count, last_layer, net_hash, x_layers, g_layers, m_layers,
    loss_balance``."""
    import pandas as pd
    seen = set()
    rows = []
    rounds = 0
    ss = np.random.SeedSequence(seed)
    while len(rows) < n and rounds < max_rounds:
        rounds += 1
        need = n - len(rows)
        child_seeds = ss.spawn(max(1, min(need, 64)))
        per = [(s, -(-need // len(child_seeds)), validation_genotype_size) for s in child_seeds]
        if workers and workers > 1:
            import multiprocessing as mp
            with mp.get_context("spawn").Pool(workers) as pool:
                chunks = pool.map(_generate_chunk, per)
        else:
            chunks = [_generate_chunk(p) for p in per]
        for chunk in chunks:
            for rec in chunk:
                if rec["net_hash"] in seen:
                    continue
                seen.add(rec["net_hash"])
                rows.append(rec)
    cols = ["code", "parameters_count", "last_layer", "net_hash", "x_layers", "g_layers", "m_layers",
            "loss_balance"]
    return pd.DataFrame(rows[:n], columns=cols)


def _generate_chunk(args):
    seed_seq, count, vgs = args
    rng = np.random.default_rng(seed_seq)
    out = []
    for _ in range(count):
        rec = generate_network(rng, vgs)
        if rec is not None:
            out.append(rec)
    return out
