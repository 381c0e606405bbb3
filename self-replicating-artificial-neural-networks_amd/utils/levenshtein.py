"""Levenshtein distance (reference uses edlib, experiment.py:16-17).  Native C++ bit-parallel
implementation (csrc/host/serann_host.cpp) with a pure-Python fallback."""
from __future__ import annotations

from typing import Sequence

from .native import load


def _py_levenshtein(a: str, b: str) -> int:
    if len(a) < len(b):
        a, b = b, a
    prev = list(range(len(b) + 1))
    for i, ca in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, cb in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb))
        prev = cur
    return prev[-1]


def levenshtein(a: str, b: str) -> int:
    h = load("serann_host")
    return h.levenshtein(a, b) if h is not None else _py_levenshtein(a, b)


def levenshtein_batch(a: Sequence[str], b: Sequence[str], threads: int = 0):
    h = load("serann_host")
    if h is not None:
        return h.levenshtein_batch(list(a), list(b), threads)
    return [_py_levenshtein(x, y) for x, y in zip(a, b)]
