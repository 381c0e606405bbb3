#!/bin/bash
# Full GPU check of the current tree: GPU test tier, smoke(), 1-GPU bench, rocprofv3 kernel statistics.
# Every GPU step has its own time limit; a fault-like exit stops the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift; local to=$1; shift
  echo "=== $name ===" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/session.log
  tail -6 "gpurun_out/$name.log" | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ]; then echo "step $name failed, stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,smoke,bench,prof}
[[ $STEPS == *tests* ]] && run gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py --steps 2 --warmup 1
if [[ $STEPS == *prof* ]]; then
  rm -rf gpurun_out/prof
  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 1
fi
exit 0
