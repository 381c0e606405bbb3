#!/bin/bash
# fused-concat check: GPU kernel + engine tests, then step time (ancestor clones / generator sample)
# with SERANN_FUSE_CONCAT on and off, interleaved in one call
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fuse_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fuse_tests.log; exit 1; }
tail -1 gpurun_out/fuse_tests.log
for fz in 1 0; do
  for af in 1.0 0.0; do
    SERANN_FUSE_CONCAT=$fz timeout -k 10 200 python scripts/bench_step.py --streams 4,1 --ancestor-frac $af > gpurun_out/fuse_${fz}_$af.log 2>&1 || { echo "step failed"; tail -5 gpurun_out/fuse_${fz}_$af.log; exit 1; }
    grep streams gpurun_out/fuse_${fz}_$af.log | sed "s/^/fuse=$fz anc=$af /"
  done
done
