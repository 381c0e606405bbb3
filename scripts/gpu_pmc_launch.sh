#!/bin/bash
# PMC counters of the slowest launch of one kernel variant in the train step of a committed population:
# bench_kernels.py times every launch, the slowest launch whose (kind, arg) matches MATCH is picked, and two
# counter passes run on that launch alone.
mkdir -p gpurun_out/pl
export TMPDIR=/tmp
R=$(pwd)
POP=${POP:-populations/bench_gen3_pop125.json}
MATCH=${MATCH:-"(2, 64016)"}
timeout -k 10 300 python3 scripts/bench_kernels.py --population-file $POP --pop 125 --out gpurun_out/pl/kb.json > gpurun_out/pl/kb.log 2>&1 || { echo "kb failed"; tail -5 gpurun_out/pl/kb.log; exit 1; }
IDX=$(python3 - "$MATCH" <<'PY'
import json, sys
rows = json.load(open("gpurun_out/pl/kb.json"))["rows"]
m = [r for r in rows if r["arg"] == sys.argv[1]]
m.sort(key=lambda r: -r["ms"])
print(m[0]["i"] if m else -1)
PY
)
echo "launch $IDX"
python3 - "$IDX" <<'PY'
import json, sys
rows = json.load(open("gpurun_out/pl/kb.json"))["rows"]
r = [x for x in rows if x["i"] == int(sys.argv[1])][0]
print(json.dumps(r))
PY
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
            "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $R/gpurun_out/pl/p$i -o run --output-format csv -- python3 scripts/bench_kernels.py --population-file $POP --pop 125 --reps 3 --only $IDX --out gpurun_out/pl/kb$i.json > gpurun_out/pl/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pl/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pl/p1 gpurun_out/pl/p2 --out gpurun_out/pl/pmc_summary.csv && cat gpurun_out/pl/pmc_summary.csv | cut -c1-600 && rm -rf gpurun_out/pl/p1 gpurun_out/pl/p2
