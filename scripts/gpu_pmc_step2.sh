#!/bin/bash
# (variant of gpu_pmc_step.sh: MAXSTEPS training steps per epoch, so each counter pass stays short)
# PMC counters of every launch of one training-step plan (scripts/bench_step.py, single stream, one epoch), one
# counter pass per run; per-kernel medians for kernels matching KRE.
#   POP=ancestor_pop125 KRE=g3_wgrad bash scripts/gpu_pmc_step.sh
mkdir -p gpurun_out/pmc_step
export TMPDIR=/tmp
POP=${POP:-ancestor_pop125}
KRE=${KRE:-g3_wgrad}
i=0
for ctrs in ${PASSES:-"FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"}; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmc_step/p$i -o run --output-format csv -- python3 \
      scripts/bench_step.py --population-file populations/$POP.json --streams 1 --epochs 1 --max-steps ${MAXSTEPS:-3} > gpurun_out/pmc_step/p$i.log 2>&1 \
      || { echo "pass $i failed"; tail -5 gpurun_out/pmc_step/p$i.log; exit 1; }
done
KRE="$KRE" python3 - <<'PY'
import csv, glob, collections, os, re
kre = re.compile(os.environ["KRE"])
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_step/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if kre.search(name):
            key = (name.split("(")[0][:70], r.get("Grid_Size", ""))
            agg[(key, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (key, ctr) in sorted(agg):
    v = sorted(agg[(key, ctr)])
    print(f"{key[0]:70s} grid {key[1]:>9s} {ctr:26s} median {v[len(v)//2]:.4g} (n={len(v)})")
PY
find gpurun_out/pmc_step -name "*.csv" -size +2M -delete
