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
from typing import List, Sequence


def lpt_partition(costs: Sequence[float], world_size: int, keys: Sequence[str] | None = None) -> List[List[int]]:
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
    heap = [(0.0, r) for r in range(world_size)]
    parts: List[List[int]] = [[] for _ in range(world_size)]
    for c, members in bundles:
        load, r = heapq.heappop(heap)
        parts[r].extend(members)
        heapq.heappush(heap, (load + c, r))
    return [sorted(p) for p in parts]


def round_robin_partition(n: int, world_size: int) -> List[List[int]]:
    return [list(range(r, n, world_size)) for r in range(world_size)]
