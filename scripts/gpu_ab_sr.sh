#!/bin/bash
# A/B of the in-tree kernels vs ab/prev: GPU kernel + engine tests, then per-launch timings of the
# ancestor population and generation times (bench.py), interleaved.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sr_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sr_tests.log; exit 1; }
tail -1 gpurun_out/sr_tests.log
for v in new prev; do
  if [ $v = prev ]; then export SERANN_NATIVE_DIR=$PWD/ab/prev; else unset SERANN_NATIVE_DIR; fi
  timeout -k 10 200 python scripts/bench_kernels.py --pop 125 --ancestor-frac 1.0 --out gpurun_out/kbsr_anc_$v.json > gpurun_out/kbsr_anc_$v.log 2>&1 || { echo "kb $v failed"; tail -5 gpurun_out/kbsr_anc_$v.log; exit 1; }
done
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export SERANN_NATIVE_DIR=$PWD/ab/prev; else unset SERANN_NATIVE_DIR; fi
    timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/absr_$v$i.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/absr_$v$i.log; exit 1; }
    tail -1 gpurun_out/absr_$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v$i', round(d['seconds_per_generation'],3), [round(g['learning_time'],3) for g in d['generations']])"
  done
done
