#!/bin/bash
# Step-time A/B of engine / planner settings given as environment assignments, interleaved (2 rounds):
#   CONFIGS="A=1 B=2;A=0" POP=populations/bench_gen3_pop125.json STREAMS=4,1 bash scripts/gpu_envab.sh
# TESTS=<pytest -k expression> first runs those GPU tests (engine + kernels) and stops on a failure.
mkdir -p gpurun_out/envab
export TMPDIR=/tmp
POP=${POP:-populations/bench_gen3_pop125.json}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q -k "$TESTS" --timeout 120 --timeout-method thread > gpurun_out/envab/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/envab/tests.log; exit 1; }
  tail -1 gpurun_out/envab/tests.log
fi
IFS=';' read -ra CFG <<< "${CONFIGS:-BASE=1}"
for round in 1 2; do
  i=0
  for c in "${CFG[@]}"; do
    i=$((i+1))
    env $c timeout -k 10 200 python scripts/bench_step.py --population-file $POP --streams ${STREAMS:-4,1} --epochs ${EPOCHS:-2} > gpurun_out/envab/r${round}_c$i.log 2>&1 || { echo "config '$c' failed"; tail -8 gpurun_out/envab/r${round}_c$i.log; exit 1; }
    grep streams= gpurun_out/envab/r${round}_c$i.log | while read -r l; do echo "[$c] $l"; done
  done
done
