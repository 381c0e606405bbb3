#!/usr/bin/env python
"""Per-launch PMC table from scripts/pmc_summary.py output (two counter passes of the same launches, see
scripts/gpu_pmc_r4_final.sh): medians over the dispatches of each (population, kernel, grid), with

    cycles    = GRBM_GUI_ACTIVE / 8 (pass 2; summed over the 8 XCDs)    us@2.1G = cycles / 2100
    mfma %    = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs)
    waves/CU  = SQ_WAVE_CYCLES x 4 / (cycles x 256 CUs)
    wait %    = SQ_WAIT_ANY / SQ_WAVE_CYCLES               issue-stall % = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
    ldsconf   = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS        L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS)
    valu/wave = SQ_INSTS_VALU / SQ_WAVES

    python scripts/pmc_table.py gpurun_out/pmc_r4_final_summary.csv --min-grid 100000
"""
import argparse
import csv
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("--min-grid", type=int, default=0, help="skip launches with fewer threads")
    a = ap.parse_args()
    groups = defaultdict(lambda: defaultdict(list))
    with open(a.summary) as f:
        for r in csv.DictReader(f):
            pop = r["pass"].rsplit("_p", 1)[0]
            key = (pop, r["kernel"].replace("void ", ""), int(r["grid"]))
            for k, v in r.items():
                if k.startswith(("SQ_", "TCC_", "GRBM_")) and v not in ("", None):
                    groups[key][k].append(float(v))
    print(f"{'pop':<9s}{'kernel':<52s}{'grid':>10s}{'us@2.1G':>9s}{'mfma%':>7s}{'waves/CU':>9s}{'wait%':>7s}"
          f"{'istall%':>8s}{'ldsconf':>8s}{'L2hit':>7s}{'valu/wave':>10s}")
    for (pop, kern, grid), c in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][2])):
        if grid < a.min_grid:
            continue
        m = {k: statistics.median(v) for k, v in c.items()}

        def g(k):
            return m.get(k, float("nan"))
        cyc = g("GRBM_GUI_ACTIVE") / 8
        wc = g("SQ_WAVE_CYCLES")
        hit, miss = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        print(f"{pop[:8]:<9s}{kern[:51]:<52s}{grid:>10d}{cyc / 2100:>9.1f}"
              f"{100 * g('SQ_VALU_MFMA_BUSY_CYCLES') / (cyc * 1024):>7.1f}{wc * 4 / (cyc * 256):>9.1f}"
              f"{100 * g('SQ_WAIT_ANY') / wc:>7.1f}{100 * g('SQ_WAIT_INST_ANY') / wc:>8.1f}"
              f"{g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_INSTS_LDS'), 1):>8.2f}{hit / max(hit + miss, 1):>7.2f}"
              f"{g('SQ_INSTS_VALU') / max(g('SQ_WAVES'), 1):>10.0f}")


if __name__ == "__main__":
    main()
