#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_kernels.py --pop 125 --out gpurun_out/bench_kernels.json > gpurun_out/kbench.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/kbench.log; exit 1; }
SERANN_WGRAD_TARGET=32 timeout -k 10 300 python scripts/bench_kernels.py --pop 125 --out gpurun_out/bench_kernels_t32.json > gpurun_out/kbench_t32.log 2>&1 || { echo "kbench32 failed"; tail -20 gpurun_out/kbench_t32.log; exit 1; }
head -3 gpurun_out/kbench_t32.log
