#!/bin/bash
# GPU-box helper: parity tests, benches of C3 / C3-Rosenbrock / C2, then the
# rocprofv3 kernel trace + FETCH/WRITE PMC passes of the C3 bench.
# Every GPU step has its own time limit; the first crash-like exit ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r01b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
crash() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.txt
crash $rc && exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail -5 $OUT/bench_c3.err; exit 1; }
tail -1 $OUT/bench_c3.json
timeout -k 10 200 python bench.py --config c3r --no-cpu-baseline > $OUT/bench_c3r.json 2> $OUT/bench_c3r.err || { echo "bench c3r failed"; exit 1; }
timeout -k 10 200 python bench.py --config c2 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail -5 $OUT/bench_c2.err; exit 1; }
tail -1 $OUT/bench_c2.json
[ -n "$NO_PROF" ] && exit 0
ARGS="--steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || { echo "kernel-trace failed"; tail -5 $OUT/kt.log; exit 1; }
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc_$pmc -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_$pmc.log 2>&1 || { echo "pmc $pmc failed"; tail -5 $OUT/pmc_$pmc.log; exit 1; }
done
python3 tools_gpu/pmc_summary.py $OUT gen_ pair_plan > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
