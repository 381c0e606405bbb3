#!/bin/bash
# kernel numerics + per-launch timing + bench for the default path and one A/B variant ($1 = SERANN_GEMM3_OFF list)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -q -x > gpurun_out/kt.log 2>&1 || { tail -25 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
timeout -k 10 300 python scripts/bench_kernels.py --out gpurun_out/bk3.json > gpurun_out/bk3.log 2>&1 || { tail -5 gpurun_out/bk3.log; exit 1; }
head -2 gpurun_out/bk3.log | tail -1
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
echo "default:"; tail -1 gpurun_out/bench.log | cut -c1-300
if [ -n "$1" ]; then
  SERANN_GEMM3_OFF=$1 timeout -k 10 300 python scripts/bench_kernels.py --out gpurun_out/bk3_off.json > gpurun_out/bk3_off.log 2>&1 || exit 1
  head -2 gpurun_out/bk3_off.log | tail -1
  SERANN_GEMM3_OFF=$1 timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_off.log 2>&1 || exit 1
  echo "off=$1:"; tail -1 gpurun_out/bench_off.log | cut -c1-300
fi
