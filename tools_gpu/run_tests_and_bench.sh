#!/bin/bash
# GPU-box helper: parity tests, then a short bench.  Stops at the first
# crash-like exit (fault / abort / segfault / timeout), continues past plain
# test failures (exit 1) so the bench line is still produced.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf --timeout 300 ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after crash-like exit"; exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"; tail -5 gpurun_out/bench.log
exit $brc
