#!/bin/bash
# A/B of the in-tree kernels against ab/prev (scripts/ab_build.sh, or a copy of the previous .so) on a
# fixed evolved population: GPU kernel + engine tests, per-launch timings and interleaved step times.
#   POP=profiles/r2_bench_population_b.json bash scripts/gpu_ab2.sh OUT
out=gpurun_out/${1:-ab2}
mkdir -p $out
export TMPDIR=/tmp
POP=${POP:-profiles/r2_bench_population_b.json}
step() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $out/$name.log; exit $rc; }; }
step tests 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread
tail -1 $out/tests.log
for v in new prev; do
  if [ $v = prev ]; then export SERANN_NATIVE_DIR=$PWD/ab/prev; else unset SERANN_NATIVE_DIR; fi
  step kb_$v 300 python scripts/bench_kernels.py --pop 125 --population-file $POP --out $out/kb_$v.json
  sed -n 2p $out/kb_$v.log | sed "s/^/$v /"
done
for i in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export SERANN_NATIVE_DIR=$PWD/ab/prev; else unset SERANN_NATIVE_DIR; fi
    step step_$v$i 250 python scripts/bench_step.py --streams 4 --population-file $POP
    grep streams= $out/step_$v$i.log | sed "s/^/$v$i /"
  done
done
