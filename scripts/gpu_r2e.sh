#!/bin/bash
# Re-entry check after a container rebuild: GPU test suite, smoke(), a 2-rank bench rehearsal (gloo
# control plane, both ranks on the one GPU: exercises the sharded bench path with the HIP engine) and
# per-launch timings of the evolved bench population.  Each GPU step has its own time limit; the first
# failure ends the script.
set -o pipefail
out=gpurun_out/${1:-r2e}
mkdir -p $out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; tail -2 $out/$name.log | cut -c1-400; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $out/$name.log; exit $rc; }; }
step gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench2 400 env SERANN_COMM_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --pop-per-gpu 32
step kbench 300 python scripts/bench_kernels.py --pop 125 --population-file profiles/r2_bench_population_b.json --out $out/bench_kernels.json
