#!/usr/bin/env python
"""Summarise a rocprofv3 --stats kernel_stats.csv: per-kernel total / share / calls / average, with the share of
the BatchNorm kernels, excluding the host<->device copies of checkpoint writes (``--exclude``)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=0, help="training steps in the profile (per-step ms column)")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--exclude", default="__amd_rocclr_copyBuffer")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.csv)) if not any(x and x in r["Name"] for x in a.exclude.split(","))]
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    bn = sum(float(r["TotalDurationNs"]) for r in rows if r["Name"].startswith("void bn_kernel"))
    per = f", {tot / 1e6 / a.steps:.2f} ms per step over {a.steps} steps" if a.steps else ""
    print(f"kernel time {tot / 1e6:.2f} ms{per} (excluding {a.exclude}); bn_kernel {100 * bn / tot:.1f} %")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        t = float(r["TotalDurationNs"])
        ps = f" {t / 1e6 / a.steps:7.3f} ms/step" if a.steps else ""
        print(f"{t / 1e6:9.2f} ms {100 * t / tot:5.1f} %{ps} calls={int(r['Calls']):5d} avg={float(r['AverageNs']) / 1e3:8.1f} us  "
              f"{r['Name'][:100]}")


if __name__ == "__main__":
    main()
