#!/bin/bash
# Round-2 evidence run: every -m gpu test, smoke(), the bench lines of C3 (with
# the CPU baseline), C2, C4 (8 islands on one GPU), C5 and C5x, rocprofv3
# kernel traces of C3 / C2 / C4 / C5 and FETCH_SIZE / WRITE_SIZE passes of C3
# and C2 (each counter its own pass).  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02z}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 $OUT/$name.err; tail -5 $OUT/$name.out; exit $rc; fi
  tail -2 $OUT/$name.out | cut -c1-400
}
[ -z "$SKIP_TESTS" ] && step pytest 900 python -u -m pytest tests -m gpu -v -rf -s --timeout 240 --timeout-method thread
[ -z "$SKIP_TESTS" ] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c3 400 python bench.py --steps 20 --warmup 5
step bench_c2 200 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline
step bench_c4 400 python bench.py --islands 8 --steps 20 --warmup 5 --no-cpu-baseline
step bench_c5 600 python bench.py --config c5 --steps 5 --warmup 2
step bench_c5x 600 python bench.py --config c5x --steps 5 --warmup 2 --no-cpu-baseline
step kt_c3 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c3 -o run --output-format csv -- python3 bench.py --steps 12 --warmup 2 --no-cpu-baseline
step kt_c2 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 20 --warmup 2 --no-cpu-baseline
step kt_c4 400 rocprofv3 --kernel-trace --stats -d $OUT/kt_c4 -o run --output-format csv -- python3 bench.py --islands 8 --steps 10 --warmup 0 --no-cpu-baseline
step kt_c5 400 rocprofv3 --kernel-trace --stats -d $OUT/kt_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline
for cfg in c3 c2; do
  for pmc in FETCH_SIZE WRITE_SIZE; do
    step pmc_${cfg}_$pmc 180 rocprofv3 --pmc $pmc -d $OUT/pmc_${cfg}_$pmc -o run --output-format csv -- python3 bench.py --config $cfg --steps 6 --warmup 1 --no-cpu-baseline
  done
done
echo "all done"
