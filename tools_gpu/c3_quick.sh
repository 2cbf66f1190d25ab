#!/bin/bash
# Quick C3/C4 check: parity tests of the float hot path, two C3 bench lines, a
# C4 line (8 islands on one GPU), the single-deme probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-full_size or checkpoint or native}" > gpurun_out/pt.log 2>&1 || { tail -5 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
show() { python3 -c "import json; d=json.load(open('gpurun_out/x.json')); print('$1', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"; }
for i in 1 2; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/x.json || exit 2; show c3; done
timeout -k 10 300 python bench.py --islands 8 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/x.json || exit 3; show c4
timeout -k 10 200 python tools_gpu/interleave_probe.py alone | grep kernel
