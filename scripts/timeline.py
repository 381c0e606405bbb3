#!/usr/bin/env python
"""Occupancy of the GPU timeline from a rocprofv3 kernel trace (``--kernel-trace``, csv).

For the window after the first ``--skip-ms`` of kernel activity (graph capture, planning copies) it reports
  * busy: the fraction of wall time with at least one kernel running (1 - idle gaps),
  * concurrency: mean number of kernels in flight while busy,
  * per kernel name: total duration, and *exposed* time -- the wall time during which that kernel was the
    only one running (what a faster version of it would save at most, to first order).
Gaps between consecutive kernels are binned, so launch / dependency latency shows up as a number.

    python scripts/timeline.py gpurun_out/tl/run_kernel_trace.csv [--skip-ms 200] [--top 25]
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name.replace("void ", ""))
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-ms", type=float, default=0.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    ev = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    ev.sort()
    t_first = ev[0][0]
    ev = [e for e in ev if e[0] >= t_first + a.skip_ms * 1e6]
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    # sweep line
    pts = []
    for i, (s, e, _) in enumerate(ev):
        pts.append((s, 1, i))
        pts.append((e, -1, i))
    pts.sort(key=lambda p: (p[0], p[1]))
    active = set()
    last = t0
    busy = 0
    conc_int = 0
    exposed = defaultdict(float)
    gaps = defaultdict(int)
    gap_total = 0
    for t, d, i in pts:
        dt = t - last
        if dt > 0:
            if active:
                busy += dt
                conc_int += dt * len(active)
                if len(active) == 1:
                    exposed[ev[next(iter(active))][2]] += dt
            else:
                gap_total += dt
                b = "<2us" if dt < 2e3 else "2-5us" if dt < 5e3 else "5-10us" if dt < 10e3 else \
                    "10-50us" if dt < 50e3 else ">=50us"
                gaps[b] += 1
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    wall = t1 - t0
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in ev:
        tot[n] += e - s
        cnt[n] += 1
    print(f"window {wall / 1e6:.2f} ms, {len(ev)} kernels; busy {100 * busy / wall:.1f} %, idle gaps "
          f"{gap_total / 1e6:.2f} ms; mean concurrency while busy {conc_int / max(busy, 1):.2f}; "
          f"sum of kernel durations {sum(tot.values()) / 1e6:.2f} ms")
    print("gaps:", dict(sorted(gaps.items())))
    print(f"{'kernel':72s} {'calls':>6s} {'sum ms':>8s} {'exposed ms':>10s} {'exp % wall':>10s}")
    for n in sorted(tot, key=lambda k: -exposed[k] - 1e-3 * tot[k])[:a.top]:
        print(f"{n:72s} {cnt[n]:6d} {tot[n] / 1e6:8.2f} {exposed[n] / 1e6:10.2f} {100 * exposed[n] / wall:9.1f}%")


if __name__ == "__main__":
    main()
