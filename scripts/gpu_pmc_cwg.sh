#!/bin/bash
# PMC counters of the isolated conv WGRAD launch (scripts/cwg_bench.py, one shape), one counter pass per run.
#   SHAPE=750,28,28,74,16,5,1 bash scripts/gpu_pmc_cwg.sh
mkdir -p gpurun_out/pmc_cwg
export TMPDIR=/tmp
SHAPE=${SHAPE:-750,28,28,74,16,5,1}
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
            "SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
            "FETCH_SIZE TCC_HIT_sum" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace -d gpurun_out/pmc_cwg/p$i -o run --output-format csv -- python3 scripts/cwg_bench.py \
      --shape $SHAPE --reps 3 > gpurun_out/pmc_cwg/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_cwg/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc_cwg/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "conv_wgrad" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = sorted(agg[k])
    print(f"{k:28s} median {v[len(v)//2]:.4g}  (n={len(v)})")
PY
find gpurun_out/pmc_cwg -name "*.csv" -size +2M -delete
