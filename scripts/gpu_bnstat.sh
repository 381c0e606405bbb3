#!/bin/bash
# BN statistics-phase block sizing A/B: kernel + engine GPU tests, BN micro-bench, step time, bench.
set -o pipefail
mkdir -p gpurun_out/bs3
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > gpurun_out/bs3/$name.log 2>&1; local rc=$?; tail -6 gpurun_out/bs3/$name.log | cut -c1-300; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 gpurun_out/bs3/$name.log; exit $rc; }; }
step tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bn 200 python scripts/bench_bn.py
step step 250 python scripts/bench_step.py --streams 4
step bench 500 python bench.py --steps 3 --warmup 1
