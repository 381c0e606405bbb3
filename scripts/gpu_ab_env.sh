#!/bin/bash
# A/B of an environment switch on the bench population: step time and per-launch table with and
# without "$AB_ENV" (e.g. AB_ENV=SERANN_GEMM3_OFF=xcd).  Usage: AB_ENV=... bash scripts/gpu_ab_env.sh OUT
set -o pipefail
out=gpurun_out/${1:-ab}
mkdir -p $out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; tail -3 $out/$name.log | cut -c1-300; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $out/$name.log; exit $rc; }; }
P=${POPFILE:-profiles/r2_bench_population.json}; [ "$P" = none ] && P=
step step_a 250 python scripts/bench_step.py ${P:+--population-file $P} --streams 4
step step_b 250 env $AB_ENV python scripts/bench_step.py ${P:+--population-file $P} --streams 4
step kern_a 300 python scripts/bench_kernels.py --pop 125 ${P:+--population-file $P} --out $out/ka.json
step kern_b 300 env $AB_ENV python scripts/bench_kernels.py --pop 125 ${P:+--population-file $P} --out $out/kb.json
python - $out <<'PY'
import json, sys
o = sys.argv[1]
a = {r["i"]: r for r in json.load(open(o + "/ka.json"))["rows"]}
b = {r["i"]: r for r in json.load(open(o + "/kb.json"))["rows"]}
print("A (default) vs B (AB_ENV): launches that differ by > 20 us")
for i in sorted(a):
    if i in b and abs(a[i]["ms"] - b[i]["ms"]) > 0.02:
        print(f"#{i:3d} {a[i]['kind']:8s} {a[i]['arg']:14s} A {a[i]['ms']:.3f}  B {b[i]['ms']:.3f}")
PY
