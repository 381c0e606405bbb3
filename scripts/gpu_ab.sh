#!/bin/bash
# A/B of environment knobs on the step time of the two fixed populations.  AB="name1:ENV=V ENV2=V;name2:..."
# (each configuration runs both populations at 4 and 1 streams; a failing step ends the script)
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
IFS=';' read -ra CFGS <<< "$AB"
for c in "${CFGS[@]}"; do
  name=${c%%:*}; envs=${c#*:}
  for pop in ${POPS:-bench_gen3_pop125 ancestor_pop125}; do
    echo "=== $name $pop ($envs)" | tee -a gpurun_out/ab/ab.log
    env $envs timeout -k 10 300 python3 scripts/bench_step.py --population-file populations/$pop.json --streams ${STREAMS:-4,1} --epochs 2 > gpurun_out/ab/${name}_$pop.log 2>&1
    rc=$?
    grep "streams=" gpurun_out/ab/${name}_$pop.log | tee -a gpurun_out/ab/ab.log
    if [ $rc -ne 0 ]; then echo "failed rc=$rc"; tail -5 gpurun_out/ab/${name}_$pop.log; exit $rc; fi
  done
done
if [ -n "$TL" ]; then
  for pop in bench_gen3_pop125 ancestor_pop125; do
    rm -rf gpurun_out/ab/trace
    env $TL timeout -k 10 300 rocprofv3 --kernel-trace -d $(pwd)/gpurun_out/ab/trace -o run --output-format csv -- python3 \
        scripts/bench_step.py --population-file populations/$pop.json --streams 1 --epochs 1 > gpurun_out/ab/tl_$pop.log 2>&1 || exit 1
    f=$(find gpurun_out/ab/trace -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/ab/${pop}_s1.csv
    rm -rf gpurun_out/ab/trace
  done
fi
exit 0
