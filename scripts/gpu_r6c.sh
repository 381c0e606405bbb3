#!/bin/bash
# Round-6 (second session) GPU call: STEPS (comma list) of
#   tests   the whole GPU suite in one pytest process (as the driver runs it)
#   sel     the GPU tests selected by TESTK
#   ab      interleaved step-time A/B of CONFIGS (env assignments, ';'-separated) on POPS (4 and 1 streams)
#   tl      single-stream kernel trace of the training step of each population in TLPOPS (env TLENV)
#   anat    per-problem GEMM anatomy (fwd / wgrad / dgrad) of the generation-15 population
#   bench   one 1-GPU bench.py run (BSTEPS timed generations after 1 warm-up)
# Every GPU step has its own time limit; a step that fails, faults or times out ends the script.
mkdir -p gpurun_out/r6c
export TMPDIR=/tmp
R=$(pwd)
STEPS=${STEPS:-tests,ab}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
step() {
  local name=$1; shift; local to=$1; shift
  echo "=== $name ===" | tee -a gpurun_out/r6c/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/r6c/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/r6c/session.log
  tail -3 "gpurun_out/r6c/$name.log" | cut -c1-400 | tee -a gpurun_out/r6c/session.log
  if grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" "gpurun_out/r6c/$name.log"; then
    echo "GPU fault in $name, stopping" | tee -a gpurun_out/r6c/session.log; exit 98
  fi
  [ $rc -eq 0 ] || exit $rc
}
has tests && step tests 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
has sel && step sel 400 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "$TESTK"
if has ab; then
  IFS=';' read -ra CFG <<< "${CONFIGS:-SERANN_GEMM3_OFF=shared;SERANN_AB=1}"
  for pop in ${POPS:-bench_r6_gen15_pop125 bench_gen3_pop125}; do
    for round in 1 2; do
      i=0
      for c in "${CFG[@]}"; do
        i=$((i+1))
        echo "--- $pop round $round [$c]" >> gpurun_out/r6c/ab.txt
        env $c timeout -k 10 200 python scripts/bench_step.py --population-file populations/$pop.json --streams ${STREAMS:-4,1} --epochs 2 > gpurun_out/r6c/ab_${pop}_r${round}_c$i.log 2>&1 || { echo "config '$c' failed"; tail -8 gpurun_out/r6c/ab_${pop}_r${round}_c$i.log; exit 1; }
        grep streams= gpurun_out/r6c/ab_${pop}_r${round}_c$i.log | while read -r l; do echo "[$pop r$round $c] $l"; done | tee -a gpurun_out/r6c/ab.txt
      done
    done
  done
fi
if has tl; then
  for pop in ${TLPOPS:-bench_r6_gen15_pop125}; do
    rm -rf gpurun_out/r6c/trace
    step tl_$pop 300 env ${TLENV:-SERANN_AB=1} rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6c/trace -o run --output-format csv -- python3 \
        scripts/bench_step.py --population-file populations/$pop.json --streams 1 --epochs 1
    f=$(find gpurun_out/r6c/trace -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/r6c/${pop}_s1.csv
    f=$(find gpurun_out/r6c/trace -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r6c/${pop}_s1_stats.csv
    rm -rf gpurun_out/r6c/trace
  done
fi
if has anat; then
  for m in fwd wgrad dgrad; do
    step anat_$m 300 python3 scripts/gemm_anatomy.py --population-file populations/bench_r6_gen15_pop125.json --mode $m --top 16
  done
fi
has bench && step bench 900 python bench.py --steps ${BSTEPS:-3} --warmup 1
# smoke: the driver's smoke() on this tree;  bench20: the driver's 1-GPU bench command (20 timed generations after 5)
has smoke && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
has bench20 && step bench20 900 python bench.py --steps 20 --warmup 5
if has prof; then
  rm -rf gpurun_out/r6c/prof
  step prof 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6c/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1
  f=$(find gpurun_out/r6c/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r6c/bench_kernel_stats.csv
  rm -rf gpurun_out/r6c/prof
fi
exit 0
