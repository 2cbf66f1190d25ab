#!/bin/bash
# Quick C2 check: native-vs-dump diagnostic at 2^20, the packed-bit parity
# tests, then bench lines of the fused kernel (8 and 4 pairs per wave) and
# of the plan + burst form.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 100 python tools_gpu/diag_c2.py 1048576 4096 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -s \
  -k "${PYTEST_K:-bits or native or full_size or var_or or varor or trajectory or generation or onemax}" > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
for e in ${C2_ENVS:-X=1 DM_BITS_PP4=1 DM_BITS_PLAN=1}; do
  env $e timeout -k 10 100 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/c2q.json || exit 2
  python3 -c "import json; d=json.load(open('gpurun_out/c2q.json')); print('$e', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['nevals_mean'])"
done
