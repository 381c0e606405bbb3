#!/bin/bash
# Round-2 evidence run: GPU test suite, smoke(), 1-GPU bench (driver's shape), step-time bench and
# rocprofv3 kernel statistics.  Usage: scripts/gpu_r2.sh OUTDIR.  Each GPU step has its own time
# limit; the first failure ends the script.
set -o pipefail
out=gpurun_out/${1:-r2}
mkdir -p $out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; tail -2 $out/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $out/$name.log; exit $rc; }; }
step gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
step step 250 python scripts/bench_step.py --streams 4,1
rm -rf $out/prof
step prof 500 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); cp "$f" $out/kernel_stats.csv
find $out/prof -name "*kernel_trace.csv" -size +30M -delete
head -25 $out/kernel_stats.csv | cut -d, -f1-5
