#!/bin/bash
# PMC counters of selected launches (IDX, comma-separated) of the train step on the bench's evolved
# population (profiles/r2_bench_population.json); one counter pass per rocprofv3 run.  Usage:
#   IDX=13,76 MATCH=convpool bash scripts/gpu_pmc2.sh OUT
out=gpurun_out/${1:-pmc}
mkdir -p $out
export TMPDIR=/tmp
IDX=${IDX:-13}
[ "$IDX" = "all" ] && IDX=""
MATCH=${MATCH:-g3_,bn_kernel,pool_,copy2d,convpool}
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $out/p$i -o run --output-format csv -- python3 scripts/bench_kernels.py --pop 125 --reps 1 --only "$IDX" --population-file ${POP:-profiles/r2_bench_population.json} --out $out/kb$i.json > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $out/p1 $out/p2 --match $MATCH --out $out/pmc_summary.csv && rm -rf $out/p1 $out/p2 && cat $out/pmc_summary.csv
