#!/bin/bash
# Round-6 (second session) measurement: single-stream kernel trace of the generation-15 population's training
# step (for scripts/launch_roofline.py) and the per-problem GEMM anatomy of its FWD / WGRAD launches.
# Every GPU step has its own time limit; a step that fails ends the script.
mkdir -p gpurun_out/r6b
export TMPDIR=/tmp
R=$(pwd)
POP=${POP:-populations/bench_r6_gen15_pop125.json}
step() {
  local name=$1; shift; local to=$1; shift
  echo "=== $name ==="
  timeout -k 10 "$to" "$@" > "gpurun_out/r6b/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -3 "gpurun_out/r6b/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
if [[ ",${STEPS:-tl,anat}," == *",tl,"* ]]; then
  rm -rf gpurun_out/r6b/trace
  step tl 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r6b/trace -o run --output-format csv -- python3 \
      scripts/bench_step.py --population-file $POP --streams 1 --epochs 1
  f=$(find gpurun_out/r6b/trace -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/r6b/gen15_s1.csv
  rm -rf gpurun_out/r6b/trace
fi
if [[ ",${STEPS:-tl,anat}," == *",anat,"* ]]; then
  for m in fwd wgrad dgrad; do
    step anat_$m 300 python3 scripts/gemm_anatomy.py --population-file $POP --mode $m --top 16
  done
fi
exit 0
