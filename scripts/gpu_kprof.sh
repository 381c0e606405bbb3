#!/bin/bash
# Per-launch kernel attribution at pop=125 + a 2-rank (gloo control plane, shared GPU) rehearsal of the
# distributed bench path.  Every GPU step has its own time limit; a failing step ends the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_kernels.py --pop 125 --out gpurun_out/bench_kernels.json > gpurun_out/kbench.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/kbench.log; exit 1; }
head -45 gpurun_out/kbench.log
SERANN_COMM_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --pop-per-gpu 40 \
  > gpurun_out/dist2.log 2>&1 || { echo "dist2 failed"; tail -30 gpurun_out/dist2.log; exit 1; }
tail -3 gpurun_out/dist2.log
