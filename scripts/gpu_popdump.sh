#!/bin/bash
# Bench-regime population: run the 1-GPU bench (driver shape), dump its last generation, then per-launch
# kernel timings and the captured step time on exactly that population.
set -o pipefail
out=gpurun_out/${1:-pop}
mkdir -p $out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; tail -2 $out/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $out/$name.log; exit $rc; }; }
step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 --dump-population $out/population.json
step kernels 300 python scripts/bench_kernels.py --pop 125 --population-file $out/population.json --out $out/kernels.json
step step 250 python scripts/bench_step.py --population-file $out/population.json --streams 4,1
