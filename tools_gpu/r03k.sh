set -o pipefail
mkdir -p gpurun_out/r03l
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "nsga2 or dominance or bitset or nondominated or front" tests > gpurun_out/r03l/pytest.out 2>&1 || { tail -30 gpurun_out/r03l/pytest.out; exit 1; }
tail -1 gpurun_out/r03l/pytest.out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -o run -d gpurun_out/r03l/dp -- python3 tools_gpu/c5_dom_probe.py 5 > gpurun_out/r03l/dp.out 2>&1 || exit 1
grep selNSGA2 gpurun_out/r03l/dp.out
timeout -k 10 200 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03l/c5.out 2>&1 || exit 1
cut -c1-400 gpurun_out/r03l/c5.out | tail -1
