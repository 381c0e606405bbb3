#!/bin/bash
# PMC counters of the heaviest launches of both fixed populations (isolated launches, scripts/bench_kernels.py):
# ancestor plan #2 (dense FWD 7160), #7 (dense DGRAD 18128: BT + BN-backward sums), #8 (dense WGRAD 64128 + fused Adam);
# generation-3 plan #23 (conv FWD halo), #224 (dense WGRAD), #272 (conv DGRAD direct), #288 / #290 (conv WGRAD halo).
# One counter pass per rocprofv3 run, each under its own time limit.
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
            "TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  for pop in ancestor_pop125:2,7,8 bench_gen3_pop125:23,224,272,288,290; do
    p=${pop%%:*}; idx=${pop##*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/pmc/${p}_p$i -o run --output-format csv -- python3 scripts/bench_kernels.py \
        --population-file populations/$p.json --pop 125 --reps 3 --only $idx --out gpurun_out/pmc/kb_${p}_$i.json > gpurun_out/pmc/${p}_p$i.log 2>&1 \
        || { echo "pass $i $p failed"; tail -5 gpurun_out/pmc/${p}_p$i.log; exit 1; }
  done
done
python3 scripts/pmc_summary.py gpurun_out/pmc/*_p1 gpurun_out/pmc/*_p2 --out gpurun_out/pmc_r4_final_summary.csv
find gpurun_out/pmc -name "*.csv" -size +2M -delete
