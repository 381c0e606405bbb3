#!/bin/bash
# A/B of the current in-tree kernels against ab/prev (built by scripts/ab_build.sh): interleaved
# step-time runs, then per-launch timings of both.
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export SERANN_NATIVE_DIR=$PWD/ab/prev; else unset SERANN_NATIVE_DIR; fi
    timeout -k 10 200 python scripts/bench_step.py --streams ${STREAMS:-4,1} > gpurun_out/ab_$v$i.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab_$v$i.log; exit 1; }
    grep streams= gpurun_out/ab_$v$i.log | sed "s/^/$v$i /"
  done
done
if [ -n "$KB" ]; then
  for v in new prev; do
    if [ $v = prev ]; then export SERANN_NATIVE_DIR=$PWD/ab/prev; else unset SERANN_NATIVE_DIR; fi
    timeout -k 10 200 python scripts/bench_kernels.py --pop 125 --out gpurun_out/kb_$v.json > gpurun_out/kb_$v.log 2>&1 || { echo "kb $v failed"; exit 1; }
    sed -n 2p gpurun_out/kb_$v.log
  done
fi
