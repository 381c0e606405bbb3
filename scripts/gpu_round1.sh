#!/bin/bash
# GPU session: tests, smoke, bench.  Stops at the first fault-like exit status.
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1; shift; local to=$1; shift
  echo "=== $name ===" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/session.log
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then echo "fault-like exit, stopping"; exit $rc; fi
  return 0
}
run info 120 python -c "import torch;print(torch.cuda.get_device_name(0), torch.cuda.device_count())"
run gputests 480 python -m pytest tests/test_gpu_engine.py -q
run smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
run bench_hip 420 python bench.py --engine hip --steps 1 --warmup 1
