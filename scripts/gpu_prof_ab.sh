#!/bin/bash
# rocprofv3 kernel statistics of the captured training step with a switch on and off (default
# SERANN_FUSE_NBN) on ancestor clones; prints the top kernels of each run.
mkdir -p gpurun_out/pab
export TMPDIR=/tmp
R=$(pwd)
SW=${SW:-SERANN_FUSE_NBN}
POPARGS=${POPARGS:---pop 125 --ancestor-frac 1.0}
for v in 1 0; do
  export $SW=$v
  rm -rf gpurun_out/pab/p$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pab/p$v -o run --output-format csv -- python3 scripts/bench_step.py $POPARGS --streams 1 --epochs 1 > gpurun_out/pab/log$v.txt 2>&1 || { echo "prof $v failed"; tail -20 gpurun_out/pab/log$v.txt; exit 1; }
  f=$(find gpurun_out/pab/p$v -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/pab/stats$v.csv
  find gpurun_out/pab/p$v -name "*_trace.csv" -delete
  grep "ms/step" gpurun_out/pab/log$v.txt
  python3 - "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/pab/stats{sys.argv[1]}.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{sys.argv[1]}: total {tot/1e6:.2f} ms")
for r in rows[:14]:
    print(f'  {float(r["TotalDurationNs"])/1e6:8.2f} ms n={r["Calls"]:>6} avg={float(r["AverageNs"])/1e3:7.1f}us {r["Name"][:90]}')
PY
done
