#!/bin/bash
# Round-2 GPU pass: every -m gpu test (with the new islands / full-size /
# bookkeeping files), then the default bench (C3), C4 with 8 islands on one
# GPU, and C2.  Stops at the first crash-like exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02a}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_X--x} -v -rf --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} -s > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" $OUT/pytest_gpu.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after crash-like exit"; exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail $OUT/bench_c3.err; exit 2; }
cat $OUT/bench_c3.json
timeout -k 10 300 python bench.py --islands 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4_8i.json 2> $OUT/bench_c4.err || { echo "bench c4 failed"; tail $OUT/bench_c4.err; exit 2; }
cat $OUT/bench_c4_8i.json
timeout -k 10 300 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail $OUT/bench_c2.err; exit 2; }
cat $OUT/bench_c2.json
exit $rc
