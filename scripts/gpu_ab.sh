#!/bin/bash
# A/B of the current in-tree kernels against ab/prev (built by scripts/ab_build.sh): interleaved
# step-time runs, then per-launch timings of both.
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export SERANN_NATIVE_DIR=$PWD/ab/prev; else unset SERANN_NATIVE_DIR; fi
    if [ -n "$BENCH" ]; then
      timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/ab_$v$i.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v$i.log; exit 1; }
      tail -1 gpurun_out/ab_$v$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v$i', round(d['seconds_per_generation'],3), [round(g['learning_time'],3) for g in d['generations']])"
    else
      timeout -k 10 200 python scripts/bench_step.py --streams ${STREAMS:-4,1} ${STEPARGS} > gpurun_out/ab_$v$i.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v$i.log; exit 1; }
      grep streams= gpurun_out/ab_$v$i.log | sed "s/^/$v$i /"
    fi
  done
done
if [ -n "$KB" ]; then
  for v in new prev; do
    if [ $v = prev ]; then export SERANN_NATIVE_DIR=$PWD/ab/prev; else unset SERANN_NATIVE_DIR; fi
    timeout -k 10 200 python scripts/bench_kernels.py --pop 125 --out gpurun_out/kb_$v.json > gpurun_out/kb_$v.log 2>&1 || { echo "kb $v failed"; exit 1; }
    sed -n 2p gpurun_out/kb_$v.log
  done
fi
