#!/bin/bash
# Evidence run for profiles/: 1-GPU bench, step-time bench, RiboAE training/encode/decode bench,
# evaluation bench, rocprofv3 kernel statistics of one bench generation.  Each GPU step has its own
# time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > gpurun_out/ev/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/ev/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -20 gpurun_out/ev/$name.log; exit $rc; }; }
step bench 500 python bench.py --steps 3 --warmup 1
step step 250 python scripts/bench_step.py --streams 4,1
step riboae 300 python scripts/bench_riboae.py
step evaluation 400 python scripts/bench_evaluation.py --genotypes 4 --per-engine 2
rm -rf gpurun_out/ev/prof
step prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1
f=$(find gpurun_out/ev/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/ev/kernel_stats.csv
find gpurun_out/ev/prof -name "*kernel_trace.csv" -size +30M -delete
head -25 gpurun_out/ev/kernel_stats.csv | cut -d, -f1-5
