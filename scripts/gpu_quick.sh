#!/bin/bash
# quick loop: kernel numerics + engine parity + per-launch timing (+ optional bench)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift; local to=$1; shift
  echo "=== $name ===" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/session.log
  tail -3 "gpurun_out/$name.log" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then echo "step failed, stopping"; exit $rc; fi
  return 0
}
run kt 400 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -q -x -k "v3 or bn or pool or engine or loss or adam"
run bk3 300 python scripts/bench_kernels.py --out gpurun_out/bk3.json
if [ "$1" = "bench" ]; then run bench 500 python bench.py --steps 2 --warmup 1; fi
