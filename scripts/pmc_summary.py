#!/usr/bin/env python
"""Condense rocprofv3 --pmc CSVs (one row per dispatch and counter) into one row per dispatch of the
kernels whose name matches --match: dispatch id, kernel, grid, counter values."""
import argparse
import csv
import glob
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--match", default="g3_,bn_kernel,pool_,copy2d")
ap.add_argument("--out", required=True)
a = ap.parse_args()
keys = [k for k in a.match.split(",") if k]
rows = defaultdict(dict)
for d in a.dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                if not any(k in name for k in keys):
                    continue
                key = (os.path.basename(d), r.get("Dispatch_Id"), name.split("(")[0][:70], r.get("Grid_Size"))
                rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
ctrs = sorted({c for v in rows.values() for c in v})
with open(a.out, "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["pass", "dispatch", "kernel", "grid"] + ctrs)
    for k, v in rows.items():
        w.writerow(list(k) + [v.get(c, "") for c in ctrs])
print(f"{len(rows)} dispatches -> {a.out}")
