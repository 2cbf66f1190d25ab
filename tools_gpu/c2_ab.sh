#!/bin/bash
# C2 pass: packed-bit parity tests, bench of the fused kernel and of the
# plan + burst form (DM_BITS_PLAN=1), kernel trace + FETCH/WRITE PMC passes
# of the fused kernel.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02g}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rf --timeout 120 --timeout-method thread -s -k "${PYTEST_K:-bits or native or trajectory or full_size or replays or generation}" > $OUT/pytest_c2.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $OUT/pytest_c2.log | tail -15
[ $rc -ne 0 ] && exit $rc
B="--config c2 --steps 50 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 python bench.py $B > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench c2 failed"; tail $OUT/bench_c2.err; exit 2; }
cat $OUT/bench_c2.json
DM_BITS_PLAN=1 timeout -k 10 200 python bench.py $B > $OUT/bench_c2_plan.json 2> $OUT/bench_c2_plan.err || { echo "bench c2 plan failed"; exit 2; }
cat $OUT/bench_c2_plan.json
DM_BITS_NOCOUNT=1 timeout -k 10 200 python bench.py $B > $OUT/bench_c2_nocount.json 2> $OUT/bench_c2_nocount.err || { echo "bench c2 nocount failed"; exit 2; }
cat $OUT/bench_c2_nocount.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/kt_c2.log 2>&1 || { echo "kt failed"; tail $OUT/kt_c2.log; exit 3; }
f=$(find $OUT/kt_c2 -name "*kernel_stats.csv" | head -1); head -8 "$f"
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/pmc_c2_$pmc -o run --output-format csv -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/pmc_c2_$pmc.log 2>&1 || { echo "pmc $pmc failed"; tail -5 $OUT/pmc_c2_$pmc.log; exit 4; }
done

if [ -n "$WITH_C3" ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo "bench c3 failed"; tail $OUT/bench_c3.err; exit 7; }
  cat $OUT/bench_c3.json
fi
if [ -n "$WITH_C4" ]; then
  timeout -k 10 300 python bench.py --islands 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4_8i.json 2> $OUT/bench_c4.err || { echo "bench c4 failed"; tail $OUT/bench_c4.err; exit 5; }
  cat $OUT/bench_c4_8i.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c4 -o run --output-format csv -- python3 bench.py --islands 8 --steps 10 --warmup 0 --no-cpu-baseline > $OUT/kt_c4.log 2>&1 || { echo "kt c4 failed"; tail $OUT/kt_c4.log; exit 6; }
  f=$(find $OUT/kt_c4 -name "*kernel_stats.csv" | head -1); head -25 "$f"
fi
echo done
