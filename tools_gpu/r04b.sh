set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 600 python -u -m pytest -v --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04b/pytest.out 2>&1; rc=$?
tail -3 gpurun_out/r04b/pytest.out
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/r04b/bench_c3.json 2> gpurun_out/r04b/bench_c3.err || exit 1
cat gpurun_out/r04b/bench_c3.json
