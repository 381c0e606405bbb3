#!/bin/bash
# Round-3 GPU session: GPU test tier, then two 1-GPU bench runs whose per-generation records must match
# (deterministic training), with every GPU step under its own time limit; a failing step stops the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift; local to=$1; shift
  echo "=== $name ===" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/session.log
  tail -4 "gpurun_out/$name.log" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step $name failed (rc=$rc), stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-kernels,engine,rest,diag,bench2}
[[ $STEPS == *kernels* ]] && run gpukernels 600 python -u -m pytest tests/test_gpu_kernels.py --maxfail=5 -q --timeout 120 --timeout-method thread
[[ $STEPS == *engine* ]] && run gpuengine 900 python -u -m pytest tests/test_gpu_engine.py --maxfail=5 -v --timeout 300 --timeout-method thread
[[ $STEPS == *rest* ]] && run gpurest 900 python -u -m pytest tests -m gpu --maxfail=5 -q --timeout 300 --timeout-method thread --ignore tests/test_gpu_kernels.py --ignore tests/test_gpu_engine.py
[[ $STEPS == *diag* ]] && run diag 600 python -u scripts/diag_grad_err.py
if [[ $STEPS == *bench2* ]]; then
  run bench_a 600 python bench.py --steps ${BSTEPS:-3} --warmup 1
  run bench_b 600 python bench.py --steps ${BSTEPS:-3} --warmup 1
fi
exit 0
