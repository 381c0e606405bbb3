#!/bin/bash
# Step time vs stream groups and hardware queues on a fixed population.
set -o pipefail
out=gpurun_out/${1:-streams2}; POP=${POP:-profiles/r2_bench_population_b.json}
mkdir -p $out
export TMPDIR=/tmp
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 250 python scripts/bench_step.py --population-file $POP --streams ${STREAMS:-4,8} > $out/q$q.log 2>&1 || { echo "q$q failed"; tail -20 $out/q$q.log; exit 1; }
  grep streams= $out/q$q.log | sed "s/^/hwq=$q /"
done
