#!/bin/bash
# A/B of a SERANN_GEMM3_OFF switch on per-launch timings of a population (twice each, interleaved).
set -o pipefail
out=gpurun_out/${1:-offab}; OFF=${OFF:-conv_wgrad_multi}; POP=${POP:-profiles/r2_bench_population_b.json}
mkdir -p $out
export TMPDIR=/tmp
for i in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export SERANN_GEMM3_OFF=$OFF; else unset SERANN_GEMM3_OFF; fi
    timeout -k 10 200 python scripts/bench_kernels.py --population-file $POP --pop 125 --out $out/kb_$v$i.json > $out/kb_$v$i.log 2>&1 || { echo "$v failed"; tail -5 $out/kb_$v$i.log; exit 1; }
    echo "$v$i $(sed -n 2p $out/kb_$v$i.log | cut -c1-90)"
  done
done
