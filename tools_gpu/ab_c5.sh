#!/bin/bash
# C5 A/B: parity tests on the default library, then bench + kernel trace for
# each library variant given in LIBS (deap_amd/libdeapmi*.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_c5}
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -z "$NO_TEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 240 --timeout-method thread -k "${PYTEST_K:-nsga2 or nondominated or dominance or front or crowding or log or dcd or nan or example}" > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
fi
for lib in ${LIBS:-deap_amd/libdeapmi.so}; do
  tag=$(basename $lib .so)
  DEAPMI_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$tag -o run --output-format csv -- python3 bench.py ${ARGS:---config c5 --steps 3 --warmup 1} > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { echo "$tag failed"; tail $OUT/bench_$tag.err; exit 2; }
  echo "== $tag"; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$tag.json
  f=$(find $OUT/kt_$tag -name "*kernel_stats.csv" | head -1); head -9 "$f" | cut -d, -f1-4 | cut -c1-150
done
