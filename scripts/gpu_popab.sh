#!/bin/bash
# Evolve a population with bench.py (dumping its last generation), then time the training step on it
# with an engine switch on and off (FLAG, e.g. SERANN_FUSE_GCHAIN).
set -o pipefail
out=gpurun_out/${1:-popab}; FLAG=${FLAG:-SERANN_FUSE_GCHAIN}; GENS=${GENS:-10}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps 2 --warmup $((GENS-2)) --dump-population $out/pop.json > $out/bench.log 2>&1 || { echo "bench failed"; tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-200
for v in 1 0; do
  env $FLAG=$v timeout -k 10 250 python scripts/bench_step.py --population-file $out/pop.json --streams 4,1 > $out/step_$v.log 2>&1 || { echo "step $v failed"; tail -20 $out/step_$v.log; exit 1; }
  grep streams= $out/step_$v.log | sed "s/^/$FLAG=$v /"
done
