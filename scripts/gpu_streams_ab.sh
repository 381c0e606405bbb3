#!/bin/bash
# Step time vs number of stream groups on the committed populations.
mkdir -p gpurun_out/st
for pop in "--pop 125 --ancestor-frac 1.0" "--population-file populations/bench_gen3_pop125.json"; do
  timeout -k 10 300 python scripts/bench_step.py $pop --streams 1,2,4,6,8 --epochs 1 2>&1 | grep "ms/step" || exit 1
done
