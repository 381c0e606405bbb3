#!/bin/bash
# Kernel tests (conv paths) + GPU engine suite + per-launch timings on the evolved population B.
set -o pipefail
out=gpurun_out/${1:-convw}
mkdir -p $out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; tail -3 $out/$name.log | cut -c1-300; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -40 $out/$name.log; exit $rc; }; }
step kernels 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread
step gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step launches 300 python scripts/bench_kernels.py --population-file profiles/r2_bench_population_b.json --pop 125 --out $out/launches.json
step step 250 python scripts/bench_step.py --population-file profiles/r2_bench_population_b.json --streams 4,1
