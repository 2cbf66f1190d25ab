#!/bin/bash
# A/B environment variants of the same library: each argument is a
# space-separated list of VAR=value settings ("" = defaults).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--steps 30 --warmup 3 --no-cpu-baseline"}
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py $ARGS > gpurun_out/abenv_$i.log 2>&1 || { echo "variant [$v] failed"; tail -5 gpurun_out/abenv_$i.log; exit 1; }
  echo "[$v]: $(tail -1 gpurun_out/abenv_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
done
