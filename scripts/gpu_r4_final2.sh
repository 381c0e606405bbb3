#!/bin/bash
# Closing session on the final round-4 tree: the GPU suite in one process and smoke() (as the driver runs them),
# single-stream kernel traces + step times of both fixed populations, then a planner-knob sweep (split-K
# target k steps, WGRAD rows per split) on both populations.  Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIPTESTS" ]; then
  STEPS=tests bash scripts/gpu_r4.sh || exit 1
  tail -1 gpurun_out/gputests.log; grep -q " passed" gpurun_out/gputests.log && ! tail -1 gpurun_out/gputests.log | grep -qE "[0-9]+ failed" || exit 1
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
STEPS=tl,step bash scripts/gpu_r4.sh || exit 1
SW="BASE=1;SERANN_SPLIT_KSTEPS=24;SERANN_SPLIT_KSTEPS=16;SERANN_WGRAD_TARGET=64;SERANN_WGRAD_TARGET=256"
CONFIGS="$SW" EPOCHS=1 bash scripts/gpu_envab.sh > gpurun_out/envab_gen3.txt 2>&1 || { tail -5 gpurun_out/envab_gen3.txt; exit 1; }
POP=populations/ancestor_pop125.json STREAMS=1 CONFIGS="$SW" EPOCHS=1 bash scripts/gpu_envab.sh > gpurun_out/envab_anc.txt 2>&1 || { tail -5 gpurun_out/envab_anc.txt; exit 1; }
cat gpurun_out/envab_gen3.txt gpurun_out/envab_anc.txt
