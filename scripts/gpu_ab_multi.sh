#!/bin/bash
# Step time (captured graph replay, 4 streams) of two fixed populations -- the bench's evolved population
# (profiles/r2_bench_population.json) and a generator sample -- under several environment switches.
# Usage: bash scripts/gpu_ab_multi.sh OUT "ENV1" "ENV2" ...   ("" = default)
set -o pipefail
out=gpurun_out/${1:-abm}; shift
mkdir -p $out
export TMPDIR=/tmp
i=0
for e in "" "$@"; do
  i=$((i+1))
  for pop in bench gen; do
    if [ $pop = bench ]; then args="--population-file profiles/r2_bench_population.json"; else args=""; fi
    timeout -k 10 200 env $e python scripts/bench_step.py $args --streams 4 --epochs 2 > $out/s${i}_$pop.log 2>&1 || { echo "failed: $e $pop"; tail -20 $out/s${i}_$pop.log; exit 1; }
    echo "[$e] $pop: $(grep -o 'ms/step=[0-9.]*' $out/s${i}_$pop.log)"
  done
done
