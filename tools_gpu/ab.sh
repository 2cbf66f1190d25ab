#!/bin/bash
# A/B the library variants on the same box: bench each (separate processes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--steps 30 --warmup 3 --no-cpu-baseline"}
for v in "$@"; do
  lib=deap_amd/libdeapmi${v}.so
  DEAPMI_LIB=$PWD/$lib timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_${v:-A}.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_${v:-A}.log; exit 1; }
  echo "variant ${v:-A}: $(tail -1 gpurun_out/ab_${v:-A}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
done
