#!/bin/bash
# Round-6 GPU session.  STEPS picks the steps (comma list); every GPU step runs under its own time limit and a
# step that faults, aborts or times out (rc not 0/1) ends the script.
#   tests                   the whole GPU suite in ONE pytest process, exactly as the driver runs it
#   sel                     the GPU tests selected by TESTK (pytest -k)
#   diag                    per-architecture gradient error report
#   bench2                  two 1-GPU bench runs whose per-generation records must match (deterministic training)
#   prof                    rocprofv3 kernel statistics of one bench generation (profiles/r3_kernel_stats.csv)
#   riboae, riboprof        RiboAE bench on the HIP trainer; rocprofv3 statistics of its training steps
#   popdump, kb             deterministic bench population dump; per-launch step table on it
#   pop1000, calib          the pop-1000 strong-scaling anchor at N=1 (dumps the population); cost-model fit on it
#   bench1                  one 1-GPU bench run
#   pop50                   BASELINE config #2: pop 50, example.json, 1 GPU
#   evaluation              seconds per evaluated genotype
#   pop50long               BASELINE config #2 at its real length: run_experiment CLI, example.json, 100 generations
#   tl                      single-stream kernel traces of both fixed populations (scripts/launch_roofline.py)
#   step                    step wall time on both fixed populations (4 and 1 streams)
#   planprof                cProfile of the 4-stream training-plan build on the generation-3 population
#   evalgeneral             BASELINE config #5: run_evaluation CLI (E = 5, R = 100, general sampler) over ~300
#                           genotypes of the pop50long experiment; dies after its first 100 pickled results
#                           (fault injection, exit 75) and is relaunched, resuming from the pickle
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
R=$(pwd)
run() {
  local name=$1; shift; local to=$1; shift
  echo "=== $name ===" | tee -a gpurun_out/session.log
  local t0=$(date +%s%N)
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc wall_ms=$(( ($(date +%s%N) - t0) / 1000000 ))" | tee -a gpurun_out/session.log
  tail -4 "gpurun_out/$name.log" | cut -c1-600 | tee -a gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step $name failed (rc=$rc), stopping"; exit $rc; fi
  # a failing test run (rc 1) may hide a GPU fault caught as an exception: nothing more runs on the GPU then
  if grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" "gpurun_out/$name.log"; then
    echo "step $name hit a GPU fault, stopping" | tee -a gpurun_out/session.log; exit 98
  fi
  return 0
}
stats() {   # keep the kernel statistics of a rocprofv3 run, drop the (large) traces
  local d=$1 out=$2
  f=$(find "$d" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$out"
  find "$d" -name "*_trace.csv" -delete
}
STEPS=${STEPS:-tests,bench1}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
has tests && run gputests 1000 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
# sel: a -k selection of the GPU suite (TESTK), one process
has sel && run sel 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "$TESTK"
has acc && run acc 500 python -u -m pytest tests/test_gpu_engine.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k as_accurate
has kern && run kern 500 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
has probe && run probe 60 ./scripts/micro/rsrc_probe
# testsall: the whole suite without -x (the conftest ends the session at a GPU fault), to see every failure
has testsall && run gputestsall 1000 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
if has diag96; then
  run diag_fused 500 python -u scripts/diag_bf16_ratio.py
  run diag_nogchain 500 env SERANN_FUSE_GCHAIN=0 python -u scripts/diag_bf16_ratio.py gchain_f64_bn_dense gchain_nobn_k9_f100 gchain_relu_conv_fanout gchain_sigmoid_stride2 convpool_bench_a
fi
has diag && run diag 600 python -u scripts/diag_grad_err.py
if has bench2; then
  run bench_a 600 python bench.py --steps ${BSTEPS:-3} --warmup 1
  run bench_b 600 python bench.py --steps ${BSTEPS:-3} --warmup 1
fi
if has prof; then
  rm -rf gpurun_out/ev/prof
  run prof 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ev/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1
  stats gpurun_out/ev/prof gpurun_out/ev/kernel_stats.csv
fi
has planprof && run planprof 300 python -u scripts/prof_plan.py --population-file populations/bench_gen3_pop125.json
has ribotest && run ribotest 400 python -u -m pytest tests/test_riboae_hip_train.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
has riboae && run riboae 400 python scripts/bench_riboae.py --engine hip
if has riboprof; then
  rm -rf gpurun_out/ev/riboprof
  run riboprof 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ev/riboprof -o run --output-format csv -- python3 scripts/bench_riboae.py --engine hip --steps 50 --warmup 5 --train-only
  stats gpurun_out/ev/riboprof gpurun_out/ev/riboae_kernel_stats.csv
fi
has popdump && run popdump 600 python bench.py --steps 3 --warmup 1 --dump-population gpurun_out/ev/pop125.json
has kb && run kb 600 python scripts/bench_kernels.py --population-file gpurun_out/ev/pop125.json --pop 125 --out gpurun_out/ev/kb_pop125.json
has pop1000 && run pop1000 1000 python bench.py --gpus 1 --pop-per-gpu 1000 --steps 2 --warmup 1 --dump-population gpurun_out/ev/pop1000.json
has calib && run calib 900 python scripts/calibrate_cost.py --population-file populations/bench_pop1000_gen2.json --measure-ranks 8 --out gpurun_out/ev/cost_model.json
has bench1 && run bench_a 600 python bench.py --steps ${BSTEPS:-3} --warmup 1
has pop50 && run pop50 600 python bench.py --gpus 1 --pop-per-gpu 50 --parameters serann/parameters/experiment/example.json --steps ${BSTEPS:-3} --warmup 1
has evaluation && run evaluation 500 python scripts/bench_evaluation.py --genotypes 4 --per-engine 2

# tl: kernel traces of the captured single-stream training step on the two fixed populations, for
# scripts/launch_roofline.py (per-launch measured vs ideal time)
if has tl; then
  mkdir -p gpurun_out/tl
  for pop in bench_gen3_pop125 ancestor_pop125; do
    rm -rf gpurun_out/tl/trace
    run tl_$pop 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tl/trace -o run --output-format csv -- python3 \
        scripts/bench_step.py --population-file populations/$pop.json --streams 1 --epochs 1
    f=$(find gpurun_out/tl/trace -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/tl/${pop}_s1.csv
    rm -rf gpurun_out/tl/trace
  done
fi
# step: wall time per step (4 streams and 1) on both fixed populations
if has step; then
  for pop in bench_gen3_pop125 ancestor_pop125; do
    run step_$pop 300 python3 scripts/bench_step.py --population-file populations/$pop.json --streams 4,1 --epochs 2
  done
fi

# EXPDIR: an experiment results directory shipped with the tree (gpurun_out/ is not pushed), e.g. the
# pop50long DB copied back for a later evalgeneral call
export SERANN_EXPERIMENT_RESULTS_DIR=${EXPDIR:-$R/gpurun_out/ev/exp}
export SERANN_SERANN_EVALUATIONS_DIR=$R/gpurun_out/ev/evals
if has pop50long; then
  mkdir -p gpurun_out/ev/exp
  run pop50long 1100 python -u evolutionary_experiment/run_experiment.py -p serann/parameters/experiment/example.json \
      --perf-log gpurun_out/ev/pop50_100gen.jsonl
fi
if has evalgeneral; then
  db=$(ls $SERANN_EXPERIMENT_RESULTS_DIR/*.sqlite | head -1)
  eid=$(basename "$db" .sqlite)
  python - "$eid" <<'PY'
import json, sys
p = json.load(open("serann/parameters/evaluation/general.json"))
p.update(experiment_id=sys.argv[1], generation_step=1, samples_per_generation=2)
json.dump(p, open("gpurun_out/ev/general_r5.json", "w"), indent=1)
PY
  echo "=== evalgeneral_cut ===" | tee -a gpurun_out/session.log
  t0=$(date +%s%N)
  SERANN_FAULT_INJECT=evaluated=100,mode=exit timeout -k 10 900 python -u serann_evaluation/run_evaluation.py \
      -p gpurun_out/ev/general_r5.json -n general_r5 > gpurun_out/evalgeneral_cut.log 2>&1
  rc=$?
  echo "rc=$rc wall_ms=$(( ($(date +%s%N) - t0) / 1000000 )) (75 = the injected death after the first pickle)" | tee -a gpurun_out/session.log
  if [ $rc -ne 75 ] && [ $rc -ne 0 ]; then echo "evalgeneral_cut failed (rc=$rc), stopping"; exit $rc; fi
  run evalgeneral 900 python -u serann_evaluation/run_evaluation.py -p gpurun_out/ev/general_r5.json -n general_r5
fi
exit 0
