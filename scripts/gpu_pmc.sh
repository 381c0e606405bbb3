#!/bin/bash
# PMC counters of selected launches of the pop=125 train step (one counter pass per rocprofv3 run)
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
IDX=${IDX:-277}
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
            "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VALU" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 scripts/bench_kernels.py --pop 125 --reps 3 --only $IDX --out gpurun_out/pmc/kb$i.json > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc/p1 gpurun_out/pmc/p2 --out gpurun_out/pmc_summary.csv && rm -rf gpurun_out/pmc
