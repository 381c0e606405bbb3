#!/bin/bash
# Chain-kernel A/B: correctness of the first variant, then per-launch timings of every variant
# (ab/NAME builds from scripts/ab_gchain.sh) on the bench population.
set -o pipefail
mkdir -p gpurun_out/abgc
export TMPDIR=/tmp
pop=profiles/r2_bench_population.json
first=1
for v in "$@"; do
  export SERANN_NATIVE_DIR=$PWD/ab/$v
  if [ $first = 1 ]; then
    timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "gchain or matches_oracle or grouping" > gpurun_out/abgc/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/abgc/tests_$v.log; exit 1; }
    tail -1 gpurun_out/abgc/tests_$v.log; first=0
  fi
  timeout -k 10 200 python scripts/bench_kernels.py --population-file $pop --pop 125 --out gpurun_out/abgc/kb_$v.json > gpurun_out/abgc/kb_$v.log 2>&1 || { echo "kb $v failed"; tail -5 gpurun_out/abgc/kb_$v.log; exit 1; }
  echo "$v $(sed -n 2p gpurun_out/abgc/kb_$v.log | cut -c1-80)"; grep "^gchain" gpurun_out/abgc/kb_$v.log
done
