#!/bin/bash
# Fused genotype chain bring-up: chain tests, full GPU suite, step time of the bench population.
set -o pipefail
out=gpurun_out/${1:-gchain}
mkdir -p $out
export TMPDIR=/tmp
pop=profiles/r2_bench_population.json
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; tail -3 $out/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -40 $out/$name.log; exit $rc; }; }
step gctests 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread -k "gchain or matches_oracle"
step gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step step 250 python scripts/bench_step.py --population-file $pop --streams 4,1
step launches 300 python scripts/bench_kernels.py --population-file $pop --pop 125 --out $out/launches.json
