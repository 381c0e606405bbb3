#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift; local to=$1; shift
  echo "=== $name ===" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/session.log
  tail -6 "gpurun_out/$name.log" | tee -a gpurun_out/session.log
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then echo "fault-like exit, stopping"; exit $rc; fi
  return 0
}
run gputests 480 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -q -x
run bench_kernels 300 python scripts/bench_kernels.py
run bench 400 python bench.py --steps 2 --warmup 1
run riboae 300 python scripts/bench_riboae.py
