#!/usr/bin/env python
"""Compare two bench_kernels.py logs launch by launch (same population and plan): per-launch time and the
per-class totals, largest differences first."""
import re
import sys
from collections import defaultdict


def parse(path):
    out = {}
    for line in open(path):
        if not line.startswith("#"):
            continue
        m = re.match(r"#\s*(\d+)\s+(\S+)\s+(\(.*?\)|\S+)\s+(\S*)\s+([\d.]+) ms", line)
        if m:
            out[int(m.group(1))] = (m.group(2) + " " + m.group(3) + " " + m.group(4), float(m.group(5)), line.strip())
    return out


a, b = parse(sys.argv[1]), parse(sys.argv[2])
cls = defaultdict(lambda: [0.0, 0.0])
for i in a:
    if i in b:
        cls[a[i][0]][0] += a[i][1]
        cls[a[i][0]][1] += b[i][1]
print(f"{'class':45s} {'A ms':>8s} {'B ms':>8s} {'B-A':>8s}")
for k, (x, y) in sorted(cls.items(), key=lambda kv: -abs(kv[1][1] - kv[1][0]))[:25]:
    print(f"{k:45s} {x:8.3f} {y:8.3f} {y - x:+8.3f}")
print(f"{'total':45s} {sum(v[0] for v in cls.values()):8.3f} {sum(v[1] for v in cls.values()):8.3f}")
