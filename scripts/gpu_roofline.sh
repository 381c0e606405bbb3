#!/bin/bash
# Roofline evidence: kernel trace + three PMC passes of the same deterministic training workload
# (bench_step on a committed population, 1 stream, MAXSTEPS steps), then scripts/roofline.py.
mkdir -p gpurun_out/rl
export TMPDIR=/tmp
R=$(pwd)
POP=${POP:-populations/bench_gen3_pop125.json}
ARGS="scripts/bench_step.py --population-file $POP --streams 1 --epochs 1 --max-steps ${MAXSTEPS:-6}"
rm -rf gpurun_out/rl/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rl/trace -o run --output-format csv -- python3 $ARGS > gpurun_out/rl/trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/rl/trace.log; exit 1; }
f=$(find gpurun_out/rl/trace -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/rl/kernel_stats.csv
find gpurun_out/rl/trace -name "*_trace.csv" -delete
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $R/gpurun_out/rl/p$i -o run --output-format csv -- python3 $ARGS > gpurun_out/rl/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/rl/p$i.log; exit 1; }
done
python3 scripts/roofline.py --stats gpurun_out/rl/kernel_stats.csv --pmc gpurun_out/rl/p1 gpurun_out/rl/p2 gpurun_out/rl/p3 \
  --csv gpurun_out/rl/roofline.csv --md gpurun_out/rl/roofline.md --title "${TITLE:-Roofline}" && rm -rf gpurun_out/rl/p1 gpurun_out/rl/p2 gpurun_out/rl/p3
