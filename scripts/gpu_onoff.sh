#!/bin/bash
# Feature on/off check: GPU kernel + engine tests, then step time (ancestor clones / generator sample)
# with the feature's env switch unset and set, in one call.  ONOFF="VAR=value" (the "off" setting).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/onoff_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/onoff_tests.log; exit 1; }
tail -1 gpurun_out/onoff_tests.log
for mode in on off; do
  for af in ${AFS:-1.0 0.0}; do
    if [ $mode = off ]; then ENVS="$ONOFF"; else ENVS=""; fi
    env $ENVS timeout -k 10 200 python scripts/bench_step.py --streams 4 --ancestor-frac $af > gpurun_out/onoff_${mode}_$af.log 2>&1 || { echo "step failed"; tail -5 gpurun_out/onoff_${mode}_$af.log; exit 1; }
    grep streams gpurun_out/onoff_${mode}_$af.log | sed "s/^/$mode anc=$af /"
  done
done
