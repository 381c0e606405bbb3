#!/bin/bash
# Iteration check: engine + kernel GPU tests, then the captured step time and the per-launch table on the
# bench's evolved population (profiles/r2_bench_population.json).  First failure ends the script.
set -o pipefail
out=gpurun_out/${1:-it}
mkdir -p $out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; tail -3 $out/$name.log | cut -c1-300; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -40 $out/$name.log; exit $rc; }; }
step tests 400 env AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread
step step 250 python scripts/bench_step.py --population-file profiles/r2_bench_population.json --streams 4,1
step kernels 300 python scripts/bench_kernels.py --pop 125 --population-file profiles/r2_bench_population.json --out $out/kernels.json
