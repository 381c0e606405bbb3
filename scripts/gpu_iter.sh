#!/bin/bash
# Iteration check: GPU kernel + engine tests, per-launch timings, 1-GPU bench (2 timed generations)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_riboae.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/iter_tests.log; exit 1; }
tail -2 gpurun_out/iter_tests.log
timeout -k 10 200 python scripts/bench_step.py --streams 4,1 > gpurun_out/step.log 2>&1 || { echo "step failed"; tail -5 gpurun_out/step.log; exit 1; }; grep streams= gpurun_out/step.log
if [ -n "$KB" ]; then timeout -k 10 200 python scripts/bench_kernels.py --pop 125 --out gpurun_out/kb_new.json > gpurun_out/kb_new.log 2>&1 || { echo "kbench failed"; tail -5 gpurun_out/kb_new.log; exit 1; }; fi
[ -n "$KB" ] && sed -n 2,8p gpurun_out/kb_new.log
if [ -z "$NOBENCH" ]; then
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/iter_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/iter_bench.log; exit 1; }
tail -1 gpurun_out/iter_bench.log | cut -c1-300
fi
