#!/bin/bash
# Kernel trace of the captured training step (bench_step, one epoch) for scripts/timeline.py.
# STREAMS (default 4), POP (population file), MAXSTEPS (steps per epoch, default all 76).
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
R=$(pwd)
POP=${POP:-populations/bench_gen3_pop125.json}
MS=""; [ -n "$MAXSTEPS" ] && MS="--max-steps $MAXSTEPS"
rm -rf gpurun_out/tl/trace
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tl/trace -o run --output-format csv -- python3 scripts/bench_step.py --population-file $POP --streams ${STREAMS:-4} --epochs 1 $MS > gpurun_out/tl/trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/tl/trace.log; exit 1; }
f=$(find gpurun_out/tl/trace -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/tl/kernel_trace.csv
rm -rf gpurun_out/tl/trace
grep "ms/step" gpurun_out/tl/trace.log
python3 scripts/timeline.py gpurun_out/tl/kernel_trace.csv --skip-ms ${SKIPMS:-300} > gpurun_out/tl/timeline.txt && cat gpurun_out/tl/timeline.txt
