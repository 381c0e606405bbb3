"""Replicated control-plane helpers: interpretation of a generation and shard planning."""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Sequence

import numpy as np

from ..genome.interpreter import InterpretResult, try_interpret
from .cost_model import organism_time


class InterpretCache:
    """LRU cache source -> InterpretResult (populations are largely clonal, so most sources repeat
    across generations)."""

    def __init__(self, image_shape=(28, 28), genotype_size=100, num_classes=10, capacity=200_000):
        self.kw = dict(image_shape=tuple(image_shape), genotype_size=genotype_size, num_classes=num_classes)
        self.capacity = capacity
        self._c: "OrderedDict[str, InterpretResult]" = OrderedDict()
        self.hits = 0
        self.misses = 0

    def __call__(self, source: str) -> InterpretResult:
        r = self._c.get(source)
        if r is not None:
            self._c.move_to_end(source)
            self.hits += 1
            return r
        self.misses += 1
        r = try_interpret(source, **self.kw)
        self._c[source] = r
        if len(self._c) > self.capacity:
            self._c.popitem(last=False)
        return r

    def prefill(self, sources: Sequence[str], comm=None):
        """Interpret every source not yet cached.  With a multi-rank communicator the unique misses
        are split over the ranks and the results all-gathered, so the replicated control plane pays
        1 / world_size of the interpretation (at pop = 1000 a generation has hundreds of new mutants,
        ~1 ms each)."""
        missing = sorted({s for s in sources if s not in self._c})
        if not missing:
            return
        if comm is None or comm.world_size == 1:
            for s in missing:
                self(s)
            return
        mine = [(s, try_interpret(s, **self.kw)) for s in missing[comm.rank::comm.world_size]]
        for part in comm.allgather_object(mine):
            for s, r in part:
                self.misses += 1
                self._c[s] = r
        while len(self._c) > self.capacity:
            self._c.popitem(last=False)


@dataclass
class GenerationPlan:
    results: List[InterpretResult]
    is_valid: np.ndarray
    is_overweight: np.ndarray
    trainable: np.ndarray          # indices of valid & not overweight organisms
    costs: np.ndarray              # per trainable organism: predicted seconds per training step (cost_model)
    arch_keys: List[str]


def plan_generation(sources: Sequence[str], cache: InterpretCache, max_parameters: float, comm=None) -> GenerationPlan:
    cache.prefill(sources, comm)
    results = [cache(s) for s in sources]
    is_valid = np.array([r.ok for r in results], dtype=bool)
    params = np.array([r.parameters_count for r in results], dtype=np.float64)
    with np.errstate(invalid="ignore"):
        is_overweight = params > max_parameters          # NaN > x is False, as in the reference
    trainable = np.nonzero(is_valid & ~is_overweight)[0]
    costs = np.array([organism_time(results[i].ir) for i in trainable], dtype=np.float64)
    keys = [results[i].ir.arch_hash() for i in trainable]
    return GenerationPlan(results, is_valid, is_overweight, trainable, costs, keys)
