#!/bin/bash
# WGRAD kernel change check: kernel numerics tests, then per-launch timings
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "wgrad or WGRAD or gemm" > gpurun_out/wtest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/wtest.log; exit 1; }
tail -2 gpurun_out/wtest.log
timeout -k 10 200 python scripts/bench_kernels.py --pop 125 --out gpurun_out/kb_new.json > gpurun_out/kb_new.log 2>&1 || { echo "kbench failed"; tail -5 gpurun_out/kb_new.log; exit 1; }
sed -n 2,14p gpurun_out/kb_new.log
