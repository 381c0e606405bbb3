#!/bin/bash
# Re-entry check after a container rebuild: full GPU test suite, smoke(), 1-GPU bench, step-time
# bench and rocprofv3 kernel statistics.  Each GPU step has its own time limit; the first failure
# ends the script.
set -o pipefail
mkdir -p gpurun_out/r10
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > gpurun_out/r10/$name.log 2>&1; local rc=$?; tail -2 gpurun_out/r10/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 gpurun_out/r10/$name.log; exit $rc; }; }
step gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python bench.py --steps 3 --warmup 1
step step 250 python scripts/bench_step.py --streams 4,1
rm -rf gpurun_out/r10/prof
step prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r10/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1
f=$(find gpurun_out/r10/prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r10/kernel_stats.csv
find gpurun_out/r10/prof -name "*kernel_trace.csv" -size +30M -delete
head -25 gpurun_out/r10/kernel_stats.csv | cut -d, -f1-5
