#!/bin/bash
mkdir -p gpurun_out/r6d
export TMPDIR=/tmp
SERANN_DGRAD_NT1_RT=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "grouped_conv or fused_act or accurate or bitwise or reproducible" > gpurun_out/r6d/sel.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6d/sel.log; exit 1; }
tail -1 gpurun_out/r6d/sel.log
for pop in bench_r6_gen15_pop125 bench_gen3_pop125; do
  for round in 1 2; do
    for c in "SERANN_AB=1" "SERANN_DGRAD_NT1_RT=8"; do
      env $c timeout -k 10 200 python scripts/bench_step.py --population-file populations/$pop.json --streams 4,1 --epochs 2 > gpurun_out/r6d/tmp.log 2>&1 || { echo "config $c failed"; tail -8 gpurun_out/r6d/tmp.log; exit 1; }
      grep streams= gpurun_out/r6d/tmp.log | sed "s/^/[$pop r$round $c] /" | tee -a gpurun_out/r6d/ab.txt
    done
  done
done
