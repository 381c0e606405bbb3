#!/bin/bash
# Phase timing + per-kernel statistics of the bench's evolved population (profiles/r2_bench_population.json).
set -o pipefail
out=gpurun_out/${1:-phases}
mkdir -p $out
export TMPDIR=/tmp
pop=profiles/r2_bench_population.json
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; tail -3 $out/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $out/$name.log; exit $rc; }; }
step phases 300 python scripts/bench_worker_phases.py --population-file $pop
step step 250 python scripts/bench_step.py --population-file $pop --streams 4,1
rm -rf $out/prof
step prof 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 scripts/bench_step.py --population-file $pop --streams 1 --epochs 1
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); cp "$f" $out/kernel_stats.csv
find $out/prof -name "*kernel_trace.csv" -size +30M -delete
