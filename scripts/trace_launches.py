#!/usr/bin/env python
"""Per-launch table of a single-stream training-step kernel trace (rocprofv3 --kernel-trace CSV), without the
plan: the trace is cut into steps at every gather_batch_kernel launch (one per training step), launches are matched
by position within the step, and each row is (position, kernel, blocks, median us over the steps) -- sorted by time.

    python scripts/trace_launches.py gpurun_out/r6c/bench_r6_gen15_pop125_s1.csv --top 40
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--step-marker", default="gather_batch_kernel")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "copyBuffer" not in r["Kernel_Name"]]
    steps, cur = [], None
    for r in rows:
        if a.step_marker in r["Kernel_Name"]:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append(r)
    n = max(set(len(s) for s in steps), key=[len(s) for s in steps].count)
    steps = [s for s in steps if len(s) == n]
    per = defaultdict(list)
    for s in steps:
        for i, r in enumerate(s):
            per[i].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    name = lambda r: re.sub(r"\(.*", "", r["Kernel_Name"])[:70]
    tab = [(statistics.median(per[i]), i, name(steps[0][i]), int(steps[0][i]["Grid_Size_X"]) // max(1, int(steps[0][i]["Workgroup_Size_X"])))
           for i in range(n)]
    total = sum(t[0] for t in tab)
    fam = defaultdict(float)
    for t in tab:
        fam[re.sub(r"<.*", "", t[2])] += t[0]
    print(f"{len(steps)} steps of {n} launches; kernel sum {total / 1e3:.2f} ms per step")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"  {v / 1e3:7.3f} ms  {100 * v / total:5.1f} %  {k}")
    print(f"\n{'us':>8} {'pos':>4} {'blocks':>7}  kernel")
    for us, i, nm, blocks in sorted(tab, reverse=True)[:a.top]:
        print(f"{us:8.1f} {i:4d} {blocks:7d}  {nm}")


if __name__ == "__main__":
    main()
