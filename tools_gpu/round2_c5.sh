#!/bin/bash
# C5 pass: NSGA-II parity tests, then bench c5 / c5x and a kernel trace of c5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02e}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread -k "${PYTEST_K:-nsga2 or nondominated or dominance or front or crowding or log or dcd or nan or example}" -s > $OUT/pytest_c5.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" $OUT/pytest_c5.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after crash-like exit"; exit $rc; fi
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "bench c5 failed"; tail $OUT/bench_c5.err; exit 2; }
cat $OUT/bench_c5.json
timeout -k 10 300 python bench.py --config c5x --steps 5 --warmup 2 > $OUT/bench_c5x.json 2> $OUT/bench_c5x.err || { echo "bench c5x failed"; tail $OUT/bench_c5x.err; exit 2; }
cat $OUT/bench_c5x.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 > $OUT/kt_c5.log 2>&1 || { echo "kt failed"; tail $OUT/kt_c5.log; exit 3; }
f=$(find $OUT/kt_c5 -name "*kernel_stats.csv" | head -1); head -25 "$f"
