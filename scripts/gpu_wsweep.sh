#!/bin/bash
# WGRAD split-policy sweep: per-launch timings for several (k-steps per split, max splits) settings
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in 128:1000000 32:64 16:32 32:16 8:24; do
  t=${cfg%%:*}; c=${cfg##*:}
  SERANN_WGRAD_TARGET=$t SERANN_WGRAD_MAXSPLIT=$c timeout -k 10 200 python scripts/bench_kernels.py --pop 125 \
    --out gpurun_out/wsweep_${t}_${c}.json > gpurun_out/wsweep_${t}_${c}.log 2>&1 || { echo "failed $cfg"; tail -5 gpurun_out/wsweep_${t}_${c}.log; exit 1; }
  sed -n 2p gpurun_out/wsweep_${t}_${c}.log
done
