#!/bin/bash
# A/B of two extension builds selected by SERANN_NATIVE_DIR: NEW (default ab/nsx) against OLD (default the
# in-tree _native), both outside the source-hash check.  GPU tests matching TESTK on NEW first, then
# interleaved captured-step timings of the ancestor clones and the bench's generation-3 population.
mkdir -p gpurun_out/abd
export TMPDIR=/tmp
NEW=${NEW:-$PWD/ab/nsx}
OLD=${OLD:-$PWD/self-replicating-artificial-neural-networks_amd/_native}
if [ -n "$TESTK" ]; then
  SERANN_NATIVE_DIR=$NEW timeout -k 10 400 python -u -m pytest tests/ -m gpu -k "$TESTK" -x -v --timeout 120 --timeout-method thread > gpurun_out/abd/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/abd/tests.log; exit 1; }
  tail -1 gpurun_out/abd/tests.log
fi
for i in 1 2; do
  for v in new old; do
    if [ $v = new ]; then D=$NEW; else D=$OLD; fi
    SERANN_NATIVE_DIR=$D timeout -k 10 200 python scripts/bench_step.py --pop 125 --ancestor-frac 1.0 --streams 4,1 --epochs 1 > gpurun_out/abd/anc_$v$i.log 2>&1 || { echo "anc $v failed"; tail -5 gpurun_out/abd/anc_$v$i.log; exit 1; }
    grep streams= gpurun_out/abd/anc_$v$i.log | sed "s/^/anc $v$i /"
    SERANN_NATIVE_DIR=$D timeout -k 10 200 python scripts/bench_step.py --population-file populations/bench_gen3_pop125.json --streams 4 --epochs 1 > gpurun_out/abd/gen3_$v$i.log 2>&1 || { echo "gen3 $v failed"; tail -5 gpurun_out/abd/gen3_$v$i.log; exit 1; }
    grep streams= gpurun_out/abd/gen3_$v$i.log | sed "s/^/gen3 $v$i /"
  done
done
