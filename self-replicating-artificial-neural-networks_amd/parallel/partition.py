"""Organism -> rank partitioning (replaces the reference's round-robin job split,
experiment.py:170-178).

Longest-processing-time-first (LPT) over a FLOP cost model balances the heavy-tailed cost
distribution (p99 ~ 18x median).  Identical architectures are kept together
when that does not unbalance the ranks (they share grouped-kernel problems).  The result is a
pure function of the inputs, so every rank computes the same partition with no communication.
Unlike the reference (9 jobs of <=112 on 8 GPUs = 2 waves), all shards run in one wave.
"""
from __future__ import annotations

import heapq
import math
from typing import List, Optional, Sequence


def lpt_partition(costs: Sequence[float], world_size: int, keys: Sequence[str] | None = None,
                  speeds: Optional[Sequence[float]] = None) -> List[List[int]]:
    """LPT over bundles of identical architectures.  ``speeds``: per-rank time multipliers (a rank with
    factor 1.2 takes 1.2x the predicted time for the same work, :class:`RankSpeedModel`); a bundle then
    goes to the rank that would FINISH it first, (load + cost) x factor -- LPT for uniform machines."""
    n = len(costs)
    if world_size <= 1:
        return [list(range(n))]
    # group identical architectures (same key) into bundles of bounded size
    order = sorted(range(n), key=lambda i: (-float(costs[i]), i))
    total = float(sum(costs)) or 1.0
    cap = total / world_size / 4.0
    bundles = []
    if keys is not None:
        by_key = {}
        for i in order:
            by_key.setdefault(keys[i], []).append(i)
        for k in sorted(by_key, key=lambda k: (-sum(costs[i] for i in by_key[k]), by_key[k][0])):
            cur, cur_cost = [], 0.0
            for i in by_key[k]:
                if cur and cur_cost + costs[i] > cap:
                    bundles.append((cur_cost, cur))
                    cur, cur_cost = [], 0.0
                cur.append(i)
                cur_cost += float(costs[i])
            if cur:
                bundles.append((cur_cost, cur))
    else:
        bundles = [(float(costs[i]), [i]) for i in order]
    bundles.sort(key=lambda b: (-b[0], b[1][0]))
    parts: List[List[int]] = [[] for _ in range(world_size)]
    if speeds is None or all(float(s) == 1.0 for s in speeds):
        heap = [(0.0, r) for r in range(world_size)]
        for c, members in bundles:
            load, r = heapq.heappop(heap)
            parts[r].extend(members)
            heapq.heappush(heap, (load + c, r))
        return [sorted(p) for p in parts]
    sp = [float(s) for s in speeds]
    load = [0.0] * world_size
    for c, members in bundles:
        r = min(range(world_size), key=lambda q: ((load[q] + c) * sp[q], q))
        parts[r].extend(members)
        load[r] += c
    return [sorted(p) for p in parts]


class RankSpeedModel:
    """Online per-rank correction of the cost model (replaces the reference's static
    round-robin split, logic/experiment.py:170-178).

    After each generation every rank knows every rank's predicted shard cost (the partition is a pure
    function of the replicated inputs) and its measured training time (it rides in the generation's
    all-gather record), so all ranks update the same factors and compute the same next partition with
    no extra communication.  A factor is the rank's measured / predicted time relative to the other
    ranks, smoothed in log space (``alpha``) and normalised to geometric mean 1: a persistently slower
    device (thermal or power capped, shared, a slower link) receives proportionally less work, while
    one-generation noise is damped.  Organism results never depend on the partition (bitwise-identical
    training in any shard), so this changes only the schedule."""

    def __init__(self, world_size: int, alpha: float = 0.7, clamp: float = 4.0):
        self.world_size = int(world_size)
        self.alpha = float(alpha)
        self.clamp = float(clamp)
        self.log_f = [0.0] * self.world_size

    @property
    def factors(self) -> List[float]:
        return [math.exp(v) for v in self.log_f]

    def update(self, predicted: Sequence[float], measured: Sequence[float]) -> List[float]:
        """``predicted[r]``: the cost model's time of rank r's shard; ``measured[r]``: its training time
        (<= 0 or a zero prediction: no information about that rank)."""
        obs = {}
        for r, (p, m) in enumerate(zip(predicted, measured)):
            if p > 0 and m > 0 and math.isfinite(m):
                obs[r] = math.log(m / p)
        if len(obs) >= 2:
            mean = sum(obs.values()) / len(obs)
            lim = math.log(self.clamp)
            for r, v in obs.items():
                # the factor that would have explained this generation, given the current factors' share
                target = max(-lim, min(lim, v - mean))
                self.log_f[r] = (1 - self.alpha) * self.log_f[r] + self.alpha * target
            g = sum(self.log_f) / self.world_size
            self.log_f = [v - g for v in self.log_f]
        return self.factors


def round_robin_partition(n: int, world_size: int) -> List[List[int]]:
    return [list(range(r, n, world_size)) for r in range(world_size)]
