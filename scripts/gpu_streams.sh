#!/bin/bash
# stream-group A/B: engine parity tests, then 1-GPU bench with 1 and 4 stream groups
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_engine.py -q -x > gpurun_out/eng.log 2>&1 || { tail -20 gpurun_out/eng.log; exit 1; }
tail -1 gpurun_out/eng.log
for s in 4 1 8; do
  SERANN_STREAMS=$s timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_s$s.log 2>&1 || { tail -5 gpurun_out/bench_s$s.log; exit 1; }
  echo "streams=$s"; tail -1 gpurun_out/bench_s$s.log | cut -c1-330
done
