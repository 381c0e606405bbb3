#!/bin/bash
# rocprofv3 kernel-trace statistics of a 1-generation bench run (graph replay included)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > gpurun_out/prof.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
exit $rc
