#!/bin/bash
# A/B of a fusion switch (default SERANN_FUSE_NBN) on the captured training step: ancestor clones (the bench's
# first generations) and the bench's evolved generation-3 population, then one bench run.
mkdir -p gpurun_out/ab
SW=${SW:-SERANN_FUSE_NBN}
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > gpurun_out/ab/$name.log 2>&1; local rc=$?; grep -h "ms/step\|metric" gpurun_out/ab/$name.log | cut -c1-300; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -20 gpurun_out/ab/$name.log; exit $rc; }; }
for v in 1 0; do
  export $SW=$v
  step anc_$v 300 python scripts/bench_step.py --pop 125 --ancestor-frac 1.0 --streams 4,1 --epochs 1
  step gen3_$v 300 python scripts/bench_step.py --population-file populations/bench_gen3_pop125.json --streams 4 --epochs 1
done
export $SW=1
step bench 400 python bench.py --steps ${BSTEPS:-3} --warmup 1
